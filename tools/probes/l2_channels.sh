#!/bin/bash
# L2 (TCC) channel balance and queueing of one sweep variant: lists the
# counters this GPU exposes, then one rocprofv3 --pmc pass (<= 4 TCC counters)
# with whichever of the per-channel request count, tag-stall and busy
# counters exist.  Usage: tools/probes/l2_channels.sh OUTDIR N SPEC
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export TMPDIR=/tmp
ROOT=$(pwd)
out=$1; n=$2; spec=$3
case "$out" in /*) ;; *) out="$ROOT/$out" ;; esac
mkdir -p "$out"
timeout -s KILL 120 python3 "$ROOT/tools/probes/list_counters.py" "$out/counters.txt" || exit $?
want=""
nt=0
for c in TCC_REQ TCC_TAG_STALL TCC_BUSY TCC_PENDING; do
  if grep -qw "$c" "$out/counters.txt" && [ $nt -lt 4 ]; then want="$want $c"; nt=$((nt+1)); fi
done
echo "counters:$want"
[ -z "$want" ] && exit 0
timeout -s KILL 90 rocprofv3 --pmc $want GRBM_GUI_ACTIVE -d "$out/p0" -o run --output-format csv -- \
  python3 "$ROOT/tools/tune.py" --n "$n" --variants "$spec" --iters 4 --rounds 1 > "$out/p0.log" 2>&1
rc=$?
echo "pmc rc=$rc"
exit $rc
