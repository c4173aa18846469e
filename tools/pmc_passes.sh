#!/bin/bash
# rocprofv3 PMC passes over tools/tune.py (one counter group per run, each under
# its own hard time limit; counter-slot limits of gfx950 respected: <= 8 SQ,
# <= 4 TCC, <= 2 TA per pass).  Counters are per dispatch: every row of the
# summary is one 1024^3 sweep (tools/summarize_rocprof.py takes the median).
# Usage: tools/pmc_passes.sh OUTDIR VARIANT [N] [DTYPE] [SET]
#   SET = default (issue, LDS, L2 / HBM bytes) | latency (L1 / TLB stalls, L2 read latency, TA / TD)
#   PMC_SHAPE="X Y Z": sweep that owned box instead of (N-2)^3 (tune.py --shape), e.g. "3 1022 1022"
#   for the 8-GPU share's boundary slab
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
ROOT=$(pwd)
out=$1; var=$2; n=${3:-1024}; dt=${4:-fp64}; set=${5:-default}
case "$out" in /*) ;; *) out="$ROOT/$out" ;; esac
mkdir -p "$out"
passes=(
  "SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS"
  "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INST_LEVEL_VMEM SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS"
  "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum"
  "TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_DRAM_sum TCC_EA0_WRREQ_64B_sum GRBM_GUI_ACTIVE"
  "FETCH_SIZE"
  "WRITE_SIZE"
)
if [ "$set" = latency ]; then
  passes=(
    "TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_UTCL1_STALL_MULTI_MISS_sum TCP_UTCL1_THRASHING_STALL_sum GRBM_GUI_ACTIVE"
    "TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_UTCL1_SERIALIZATION_STALL_sum"
    "TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum SQ_WAVE_CYCLES SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_VMEM"
  )
fi
i=0
for p in "${passes[@]}"; do
  timeout -s KILL 90 rocprofv3 --pmc $p -d "$out/p$i" -o run --output-format csv -- \
    python3 "$ROOT/tools/tune.py" --n "$n" --dtype "$dt" --variants "$var" --iters 4 --rounds 1 \
    ${PMC_SHAPE:+--shape $PMC_SHAPE} > "$out/p$i.log" 2>&1
  rc=$?
  echo "pass $i rc=$rc"
  [ $rc -ne 0 ] && exit $rc
  i=$((i+1))
done
exit 0
