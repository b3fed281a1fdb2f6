#!/bin/bash
# PMC counters for conv shapes (kernel-trace + pmc only; no sys/hip tracing).
# usage: SHAPES="256x14x14x256x3x3x1x1 ..." bash scripts/pmc_conv.sh [outdir]
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=$R/gpurun_out/${1:-pmc}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > $O/counters_list.txt 2>&1 || true
pick() { python3 - "$O/counters_list.txt" "$@" <<'PY'
import sys, re
txt = open(sys.argv[1]).read()
have = [c for c in sys.argv[2:] if re.search(r'\b' + re.escape(c) + r'\b', txt)]
print(" ".join(have))
PY
}
SET1=$(pick SQ_WAVES SQ_BUSY_CU_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE)
SET2=$(pick TA_BUSY_avr TA_DATA_STALLED_BY_TC_CYCLES_sum TD_TC_STALL_sum)
SET3=$(pick SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_INST_LEVEL_VMEM SQ_LDS_BANK_CONFLICT SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_LDS_IDX_ACTIVE)
SET4=$(pick SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_INSTS_MFMA)
SET5=$(pick TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCC_EA0_RDREQ_sum)
for shape in ${SHAPES:-256x14x14x256x3x3x1x1 64x56x56x64x3x3x1x1}; do
  i=0
  for S in "$SET1" "$SET2" "$SET3" "$SET4" "$SET5"; do
    i=$((i+1))
    [ -z "$S" ] && continue
    timeout -k 10 200 rocprofv3 --kernel-trace --pmc $S --output-format csv -d $O/${shape}_s$i -o run -- python3 $R/scripts/bench_conv.py --only $shape --iters 3 $BENCH_ARGS > $O/${shape}_s$i.log 2>&1
    rc=$?; echo "$shape set$i rc=$rc" >> $O/status.txt
    [ $rc -eq 0 ] || exit $rc
  done
done
exit 0
