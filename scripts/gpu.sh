#!/bin/bash
# One parameterised GPU-box runner (replaces the round-1 one-off gpu_s*.sh replay scripts).
#
#   bash scripts/gpu.sh TAG STEP [STEP ...]
#
# Every step runs under its own `timeout -k 10`, logs to gpurun_out/TAG_<step>.log and appends
# "<step> rc=N" to gpurun_out/TAG_status.txt; the first failing step ends the call (no GPU work
# after a fault, abort or time limit).  Steps:
#   pytest:<file>[::expr]  python -u -m pytest <file> -m gpu -x -v [-k "expr", commas read as spaces]
#   pytest-all             every GPU test
#   smoke                  __graft_entry__.smoke()
#   bench[:args]           python bench.py <args with , as separator>  (bench:--force-comm,--steps,20)
#   prof[:args]            rocprofv3 --kernel-trace --stats of bench.py <args>  -> gpurun_out/TAG_prof
#   trace[:args]           rocprofv3 --kernel-trace --hip-trace of bench.py <args>   -> gpurun_out/TAG_trace
#   pmc:<counters>[:args]  one rocprofv3 --pmc pass over bench.py <args>          -> gpurun_out/TAG_pmc_N
#   py:<script>[:args]     python -u <script> <args>
#   pmcpy:<ctrs>:<script>[:args]  one rocprofv3 --pmc pass over python <script> <args>  -> TAG_pmc_N
#   exe:<binary>[:args]    a program built in-tree beforehand (e.g. build/prio_repro)
#   env:VAR=VALUE          export VAR for the steps after it (env:VAR= unsets it)
set -o pipefail
TAG=${1:?tag}; shift
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
O="$R/gpurun_out"; mkdir -p "$O"
npmc=0
nstep=0
run() {  # run NAME SECONDS cmd...  (logs: TAG_<NN>_<name>.log, NN = step number)
  nstep=$((nstep+1))
  local name=$(printf "%02d_%s" $nstep "$1") secs=$2; shift 2
  echo "[$(date +%T)] $name: $*" | tee -a "$O/${TAG}_status.txt"
  timeout -k 10 "$secs" "$@" > "$O/${TAG}_${name}.log" 2>&1
  local rc=$?
  echo "[$(date +%T)] $name rc=$rc" | tee -a "$O/${TAG}_status.txt"
  tail -n 3 "$O/${TAG}_${name}.log"
  return $rc
}
for st in "$@"; do
  kind=${st%%:*}; rest=""; [ "$kind" != "$st" ] && rest=${st#*:}
  case $kind in
    pytest)
      f=${rest%%::*}; k=""; [ "$f" != "$rest" ] && k=${rest#*::}; k=${k//,/ }
      n=$(basename "$f" .py)
      if [ -n "$k" ]; then
        run "pytest_$n" 900 python -u -m pytest "$f" -m gpu -x -v --timeout 240 --timeout-method thread -k "$k" || exit 1
      else
        run "pytest_$n" 900 python -u -m pytest "$f" -m gpu -x -v --timeout 240 --timeout-method thread || exit 1
      fi ;;
    pytest-all)
      run pytest_all 1100 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread || exit 1 ;;
    smoke)
      run smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" || exit 1 ;;
    bench)
      args=${rest//,/ }
      run "bench_$(echo "$args" | tr -cd 'a-z0-9-' | cut -c1-40)" 400 python -u bench.py $args || exit 1 ;;
    prof)
      args=${rest//,/ }
      ( cd /tmp && export TMPDIR=/tmp && run prof 500 rocprofv3 --kernel-trace --stats --output-format csv \
          -d "$O/${TAG}_prof" -o run -- python3 "$R/bench.py" $args ) || exit 1
      nstep=$((nstep+1)) ;;  # run() counted inside the subshell
    trace)  # kernel + HIP API trace (host launch time vs kernel start), no counters
      args=${rest//,/ }
      ( cd /tmp && export TMPDIR=/tmp && run trace 500 rocprofv3 --kernel-trace --hip-trace --output-format csv \
          -d "$O/${TAG}_trace" -o run -- python3 "$R/bench.py" $args ) || exit 1
      nstep=$((nstep+1)) ;;
    pmc)
      ctr=${rest%%:*}; args=""; [ "$ctr" != "$rest" ] && args=${rest#*:}; args=${args//,/ }
      npmc=$((npmc+1))
      ( cd /tmp && export TMPDIR=/tmp && run "pmc_$npmc" 300 rocprofv3 --pmc ${ctr//+/ } --kernel-trace \
          --output-format csv -d "$O/${TAG}_pmc_$npmc" -o run -- python3 "$R/bench.py" $args ) || exit 1
      nstep=$((nstep+1)) ;;  # run() counted inside the subshell
    pmcpy)
      ctr=${rest%%:*}; r2=${rest#*:}; s=${r2%%:*}; args=""; [ "$s" != "$r2" ] && args=${r2#*:}; args=${args//,/ }
      npmc=$((npmc+1))
      ( cd /tmp && export TMPDIR=/tmp && run "pmc_$npmc" 300 rocprofv3 --pmc ${ctr//+/ } --kernel-trace \
          --output-format csv -d "$O/${TAG}_pmc_$npmc" -o run -- python3 "$R/$s" $args ) || exit 1
      nstep=$((nstep+1)) ;;
    py)
      s=${rest%%:*}; args=""; [ "$s" != "$rest" ] && args=${rest#*:}; args=${args//,/ }
      run "py_$(basename "$s" .py)" 900 python -u "$s" $args || exit 1 ;;
    exe)
      b=${rest%%:*}; args=""; [ "$b" != "$rest" ] && args=${rest#*:}; args=${args//,/ }
      run "exe_$(basename "$b")" 300 "./$b" $args || exit 1 ;;
    env)
      var=${rest%%=*}; val=${rest#*=}
      if [ -n "$val" ]; then export "$var=$val"; else unset "$var"; fi
      echo "[$(date +%T)] env $var=$val" | tee -a "$O/${TAG}_status.txt" ;;
    *) echo "unknown step $st"; exit 2 ;;
  esac
done
exit 0
