#!/bin/bash
# PMC passes over the default C2 add path (tools/microbench.py pa2) -> gpurun_out/pmc_pa2/
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/pmc_pa2
rm -rf "$O"; mkdir -p "$O"
export TMPDIR=/tmp
cd /tmp || exit 1
rocprofv3 --list-avail > "$O/avail.txt" 2>&1 || true
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INST_CYCLES_SALU GRBM_GUI_ACTIVE" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_FLAT TCC_EA0_WRREQ_sum TCC_EA0_RDREQ_sum"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set --kernel-trace --output-format csv -d "$O/p$i" -o p -- python3 "$R/tools/microbench.py" pa2 --keys 100000000 > "$O/p$i.log" 2>&1 || echo "pass $i failed" >> "$O/fail.txt"
  f=$(find "$O/p$i" -name "*counter_collection.csv" | head -1)
  [ -n "$f" ] && { head -1 "$f"; grep -E "rbx::" "$f"; } > "$O/p${i}_rows.csv"
  rm -rf "$O/p$i"
done
echo done
