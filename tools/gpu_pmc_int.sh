# SQ counter passes over one InT cell forward + backward (B=256, T=8 bf16,
# tools/pmc_cell.py): MFMA busy and wait split per kernel (TAG names outputs)
set -o pipefail
export TMPDIR=/tmp
TAG=${TAG:-ip}
mkdir -p gpurun_out
i=0
for ctrs in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA" \
            "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -k 10 -s KILL 300 rocprofv3 --pmc $ctrs --kernel-trace --output-format csv -d gpurun_out/${TAG}_pmc$i -o run -- python3 tools/pmc_cell.py > gpurun_out/${TAG}_pmc$i.log 2>&1
  r=$?; echo PASS$i $r; [ $r -eq 0 ] || { tail -5 gpurun_out/${TAG}_pmc$i.log; exit $r; }
done
python tools/pmc_summary.py gpurun_out/${TAG}_pmc_summary.json gpurun_out/${TAG}_pmc1 gpurun_out/${TAG}_pmc2 --rm > gpurun_out/${TAG}_pmc_summary.txt
python3 - gpurun_out/${TAG}_pmc_summary.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print(f"{'kernel':44s} {'MFMA busy/SIMD':>15s} {'wait_any':>9s} {'wait_inst':>9s} {'active':>7s}")
for k, c in sorted(d.items()):
    if not k.startswith("k_") or not c.get("SQ_INSTS_MFMA"):
        continue
    simd_cycles = 1024 * c["GRBM_GUI_ACTIVE"] / 8          # 256 CUs x 4 SIMDs, GUI summed over 8 XCDs
    wc = c["SQ_WAVE_CYCLES"]
    print(f"{k:44s} {c['SQ_VALU_MFMA_BUSY_CYCLES'] / simd_cycles:15.3f} {c['SQ_WAIT_ANY'] / wc:9.3f} "
          f"{c['SQ_WAIT_INST_ANY'] / wc:9.3f} {c['SQ_ACTIVE_INST_ANY'] / wc:7.3f}")
PY
