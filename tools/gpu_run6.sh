set -o pipefail
export TMPDIR=/tmp
MASKS=0,8,16,32,56,4 timeout -k 10 300 python tools/ablate.py > gpurun_out/ablate6.log 2>&1
echo ABL_EXIT $?
cat gpurun_out/ablate6.log
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD --output-format csv -d gpurun_out/pmc6a -o run -- python3 tools/pmc_cell.py > gpurun_out/pmc6a.log 2>&1
echo PMC_A $?
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INSTS_VALU_TRANS_F32 --output-format csv -d gpurun_out/pmc6b -o run -- python3 tools/pmc_cell.py > gpurun_out/pmc6b.log 2>&1
echo PMC_B $?
