# SQ / cache counter passes over one ConvLSTM cfg3 step (k=7, B=256, T=64 bf16):
# where the conv, weight-gradient and point-wise kernels spend their cycles.
set -o pipefail
export TMPDIR=/tmp
TAG=${TAG:-lp}
mkdir -p gpurun_out
i=0
for ctrs in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA" \
            "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VMEM SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_LDS" \
            "TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 -s KILL 300 rocprofv3 --pmc $ctrs --kernel-trace --output-format csv -d gpurun_out/${TAG}_pmc$i -o run -- python3 tools/bench_convlstm.py --video --filt 7 --no-cpu-baseline --steps 1 --warmup 1 > gpurun_out/${TAG}_pmc$i.log 2>&1
  r=$?; echo PASS$i $r; [ $r -eq 0 ] || { tail -5 gpurun_out/${TAG}_pmc$i.log; exit $r; }
done
python tools/pmc_summary.py gpurun_out/${TAG}_pmc_summary.json gpurun_out/${TAG}_pmc1 gpurun_out/${TAG}_pmc2 gpurun_out/${TAG}_pmc3 --rm > gpurun_out/${TAG}_pmc_summary.txt
cat gpurun_out/${TAG}_pmc_summary.txt
