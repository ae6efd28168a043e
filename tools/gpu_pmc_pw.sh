# PMC passes over one fwd+bwd of the cell (B=256, T=8): where the point-wise kernels stall
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
# libraries are prebuilt in-tree
i=0
for ctrs in "SQ_WAVES SQ_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" \
            "SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU" \
            "SQ_INST_LEVEL_VMEM SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_LDS_IDX_ACTIVE SQ_INSTS_MFMA SQ_ACTIVE_INST_SCA"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $ctrs --kernel-trace --output-format csv -d gpurun_out/pmcpw$i -o run -- python3 tools/pmc_cell.py > gpurun_out/pmcpw$i.log 2>&1
  r=$?; echo PASS$i $r; [ $r -eq 0 ] || { tail -5 gpurun_out/pmcpw$i.log; exit $r; }
done
python tools/pmc_summary.py gpurun_out/pmcpw_summary.json gpurun_out/pmcpw1 gpurun_out/pmcpw2 gpurun_out/pmcpw3 > gpurun_out/pmcpw_summary.txt
cat gpurun_out/pmcpw_summary.txt
