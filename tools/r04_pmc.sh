#!/bin/bash
# Round 4: SQ counter passes of the symbol pass, the tree against variant libraries, SF7 and
# SF12 workloads (tools/prof_workload.py).  usage: tools/r04_pmc.sh [variant...]
set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" || exit 2
OUT=gpurun_out/pmc4
mkdir -p $OUT
V=$PWD/lora-sdr-lightweight-standalone-library-_amd/lora_phy_amd/lib/variants
G1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU"
G2="SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_VMEM"
G3="GRBM_GUI_ACTIVE SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_SCA SQ_INSTS_VALU_TRANS_F32 SQ_ACTIVE_INST_MISC SQ_IFETCH SQ_INSTS_BRANCH SQ_LDS_IDX_ACTIVE"
for v in default "$@"; do
  if [ $v = default ]; then lib=""; else lib=$V/$v.so; fi
  g=0
  for grp in "$G1" "$G2" "$G3"; do
    g=$((g+1))
    for cfg in "7 none 15625 2" "12 none 4000 2"; do
      sf=${cfg%% *}
      echo "== $v g$g sf$sf $(date +%T)"
      LORA_MI355X_LIB=$lib timeout -s KILL 150 rocprofv3 --pmc $grp --output-format csv -d $OUT/${v}_g${g}_sf$sf -o run -- python3 tools/prof_workload.py $cfg > $OUT/${v}_g${g}_sf$sf.log 2>&1 || { echo "pmc pass failed"; tail -3 $OUT/${v}_g${g}_sf$sf.log; exit 2; }
    done
  done
done
python3 tools/pmc_table.py $OUT > $OUT/table.txt; cat $OUT/table.txt
echo "== done $(date +%T)"
