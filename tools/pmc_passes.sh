#!/bin/bash
# rocprofv3 PMC passes over tools/tune.py (one counter group per run, each under
# its own hard time limit).  Usage: tools/pmc_passes.sh OUTDIR VARIANT [N] [DTYPE]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
ROOT=$(pwd)
out=$1; var=$2; n=${3:-1024}; dt=${4:-fp64}
case "$out" in /*) ;; *) out="$ROOT/$out" ;; esac
mkdir -p "$out"
passes=(
  "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU"
  "SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE GRBM_COUNT"
  "FETCH_SIZE"
  "WRITE_SIZE"
)
i=0
for p in "${passes[@]}"; do
  timeout -s KILL 90 rocprofv3 --pmc $p -d "$out/p$i" -o run --output-format csv -- \
    python3 "$ROOT/tools/tune.py" --n "$n" --dtype "$dt" --variants "$var" --iters 4 --rounds 1 > "$out/p$i.log" 2>&1
  rc=$?
  echo "pass $i rc=$rc"
  [ $rc -ne 0 ] && exit $rc
  i=$((i+1))
done
exit 0
