#!/bin/bash
# The one GPU runner (replaces round 1-2's one-off tools/gpu_*.sh scripts).
#
#   gpurun --timeout 1200 -- bash tools/gpu_run.sh OUT 'STEP ARGS' ['STEP ARGS' ...]
#
# Every step runs under its own time limit; the script stops at the first
# step that fails (GPU fault, abort, time limit) and runs nothing after it.
# OUT is a directory under gpurun_out/ (created).  Steps:
#
#   build                   __graft_entry__.build() on the box (a fresh configure: the checkout
#                           path differs from the one the shipped build/ was configured in)
#                                                                          -> OUT/build.log
#   suite [PYTEST ARGS]     python -m pytest -m gpu (default: tests/)       -> OUT/pytest.log
#   smoke                   __graft_entry__.smoke()                        -> OUT/smoke.log
#   bench [BENCH ARGS]      python bench.py ARGS (1 GPU, or --gpus N self-launch)
#                                                                          -> OUT/bench<i>.json
#   rccl [N] [BENCH ARGS]   N (default 2) ranks of bench.py sharing the one GPU over real RCCL
#                           (every rank its own NCCL_HOSTID: RCCL's network transport on loopback),
#                           each rank started by this shell                -> OUT/rccl<i>.json
#   rccltrace [N] [ARGS]    the same, every rank under rocprofv3 --kernel-trace, then
#                           tools/trace_overlap.py                         -> OUT/rccltrace<i>/, .md
#   stats [BENCH ARGS]      rocprofv3 --kernel-trace --stats of bench.py    -> OUT/stats<i>/
#   tune [TUNE ARGS]        python tools/tune.py ARGS                       -> OUT/tune<i>.log
#   proxy [PROXY ARGS]      python tools/rank_proxy.py ARGS                 -> OUT/proxy<i>.json
#   proxytrace [PROXY ARGS] the same under rocprofv3 --kernel-trace          -> OUT/proxytrace<i>/
#   pmc VARIANT [N] [DTYPE] tools/pmc_passes.sh (one counter group per run) -> OUT/pmc<i>/
#   py SCRIPT [ARGS]        any python script                              -> OUT/py<i>.log
#   exe BINARY [ARGS]       a probe binary, 120 s limit                     -> OUT/exe<i>.log
#   sh COMMAND...           a shell command (keep GPU work under its own timeout)
#   env VAR=VALUE ...       export for the later steps
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
ROOT=$(pwd)
OUT=$1; shift
case "$OUT" in /*) ;; *) OUT="$ROOT/$OUT" ;; esac
mkdir -p "$OUT"
i=0

fail() { echo "step $i ($1) failed rc=$2"; exit "$2"; }

rccl_ranks() {  # $1 = n, $2 = tag, $3 = 1 to trace, rest = bench args
  local n=$1 tag=$2 trace=$3; shift 3
  local port=$((20000 + RANDOM % 20000)) pids=() r rc=0
  for ((r = 0; r < n; r++)); do
    local pre=()
    [ "$trace" = 1 ] && pre=(rocprofv3 --kernel-trace --output-format csv -d "$OUT/$tag/rank$r" -o trace --)
    RANK=$r LOCAL_RANK=$r WORLD_SIZE=$n LOCAL_WORLD_SIZE=$n GROUP_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=$port \
      NCCL_HOSTID=heat3d-run-rank$r NCCL_SOCKET_IFNAME=lo \
      timeout -k 10 "${RANK_TIMEOUT:-400}" "${pre[@]}" python3 -u bench.py --gpus "$n" --comm rccl --watchdog 120 "$@" \
      > "$OUT/$tag.rank$r.log" 2>&1 &
    pids+=($!)
  done
  for p in "${pids[@]}"; do
    wait "$p" || rc=$?
  done
  grep -h '^{' "$OUT/$tag.rank0.log" > "$OUT/$tag.json"
  cut -c1-220 "$OUT/$tag.json"
  return $rc
}

for step in "$@"; do
  i=$((i + 1))
  eval "a=($step)"  # quotes inside a step group words, e.g. 'suite tests/ -k "a or b"' 
  name=${a[0]}
  args=("${a[@]:1}")
  echo "== step $i: $step"
  case "$name" in
    build)
      timeout -k 10 900 python3 -c "import __graft_entry__ as g; g.build()" > "$OUT/build$i.log" 2>&1 \
        || { rc=$?; tail -30 "$OUT/build$i.log"; fail build $rc; }
      tail -2 "$OUT/build$i.log" ;;
    suite)
      [ ${#args[@]} -eq 0 ] && args=(tests/)
      timeout -k 10 1000 python3 -u -m pytest -x -q --durations 8 --timeout 200 --timeout-method thread -m gpu \
        "${args[@]}" > "$OUT/pytest$i.log" 2>&1 || { rc=$?; tail -30 "$OUT/pytest$i.log"; fail suite $rc; }
      tail -2 "$OUT/pytest$i.log" ;;
    smoke)
      timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke$i.log" 2>&1 \
        || { rc=$?; tail -20 "$OUT/smoke$i.log"; fail smoke $rc; }
      tail -2 "$OUT/smoke$i.log" ;;
    bench)
      timeout -k 10 600 python3 -u bench.py "${args[@]}" > "$OUT/bench$i.json" 2> "$OUT/bench$i.err" \
        || { rc=$?; tail -20 "$OUT/bench$i.err"; fail bench $rc; }
      cut -c1-220 "$OUT/bench$i.json" ;;
    rccl|rccltrace)
      n=2
      if [[ ${args[0]:-} =~ ^[0-9]+$ ]]; then n=${args[0]}; args=("${args[@]:1}"); fi
      tr=0; [ "$name" = rccltrace ] && tr=1
      rccl_ranks "$n" "$name$i" "$tr" "${args[@]}" || { rc=$?; tail -20 "$OUT/$name$i".rank*.log; fail "$name" $rc; }
      if [ $tr = 1 ]; then
        python3 tools/trace_overlap.py "$OUT/$name$i" > "$OUT/$name$i.md" || fail trace_overlap $?
        grep -E '^\| (interior|boundary|rccl|check|other) ' "$OUT/$name$i.md"
      fi ;;
    stats)
      timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/stats$i" -o run -- \
        python3 bench.py "${args[@]}" > "$OUT/stats$i.log" 2>&1 || { rc=$?; tail -20 "$OUT/stats$i.log"; fail stats $rc; }
      python3 tools/summarize_rocprof.py "$OUT/stats$i" > "$OUT/stats$i.md"; grep -h '^{' "$OUT/stats$i.log" | cut -c1-200 ;;
    tune)
      timeout -k 10 600 python3 -u tools/tune.py "${args[@]}" > "$OUT/tune$i.log" 2>&1 \
        || { rc=$?; tail -20 "$OUT/tune$i.log"; fail tune $rc; }
      tail -25 "$OUT/tune$i.log" ;;
    proxy)
      timeout -k 10 400 python3 -u tools/rank_proxy.py "${args[@]}" > "$OUT/proxy$i.json" 2>&1 \
        || { rc=$?; tail -20 "$OUT/proxy$i.json"; fail proxy $rc; }
      tail -1 "$OUT/proxy$i.json" | cut -c1-300 ;;
    proxytrace)
      timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d "$OUT/proxytrace$i" -o trace -- \
        python3 -u tools/rank_proxy.py "${args[@]}" > "$OUT/proxytrace$i.log" 2>&1 \
        || { rc=$?; tail -20 "$OUT/proxytrace$i.log"; fail proxytrace $rc; }
      tail -1 "$OUT/proxytrace$i.log" | cut -c1-300 ;;
    pmc)
      bash tools/pmc_passes.sh "$OUT/pmc$i" "${args[@]}" || fail pmc $?
      echo "pmc done" ;;
    py)
      timeout -k 10 600 python3 -u "${args[@]}" > "$OUT/py$i.log" 2>&1 || { rc=$?; tail -20 "$OUT/py$i.log"; fail py $rc; }
      tail -20 "$OUT/py$i.log" ;;
    exe)
      timeout -k 5 120 "${args[@]}" > "$OUT/exe$i.log" 2>&1 || { rc=$?; tail -20 "$OUT/exe$i.log"; fail exe $rc; }
      tail -30 "$OUT/exe$i.log" ;;
    sh)
      bash -c "${args[*]}" || fail sh $? ;;
    env)
      export "${args[@]}" ;;
    *)
      echo "unknown step '$name'"; exit 2 ;;
  esac
done
echo "all $i steps ok"
