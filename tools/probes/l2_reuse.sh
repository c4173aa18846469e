#!/bin/bash
# L2 reuse of the tile overlap vs the x plan: HBM read requests per sweep for
# kernel specs that differ only in their x segmentation (one rocprofv3 --pmc
# pass per spec, 4 TCC counters + GRBM), then interleaved timing of the same
# specs.  Usage: [DTYPE=fp32] tools/probes/l2_reuse.sh OUTDIR N SPEC...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export TMPDIR=/tmp
ROOT=$(pwd)
out=$1; n=$2; shift 2
dt=${DTYPE:-fp64}
case "$out" in /*) ;; *) out="$ROOT/$out" ;; esac
mkdir -p "$out"
i=0
for v in "$@"; do
  timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE \
    -d "$out/p$i" -o run --output-format csv -- \
    python3 "$ROOT/tools/tune.py" --n "$n" --dtype "$dt" --variants "$v" --iters 4 --rounds 1 > "$out/p$i.log" 2>&1
  rc=$?
  echo "pmc $i $v rc=$rc"
  [ $rc -ne 0 ] && exit $rc
  i=$((i+1))
done
timeout -k 10 300 python3 "$ROOT/tools/tune.py" --n "$n" --dtype "$dt" --iters 6 --rounds 3 --variants "$@" > "$out/tune.log" 2>&1
rc=$?
echo "tune rc=$rc"
exit $rc
