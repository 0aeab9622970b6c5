#!/bin/bash
# The one GPU runner (round 3 on): a gpurun call runs `tools/gpu.sh <tag> <step> [<step> ...]`; every step
# writes its log under gpurun_out/<tag>/, runs under its own time limit, and the first failing step ends
# the call (no further GPU work after a failure, a fault or a time limit).
#
# Steps (an argument "name" or "name:args", args split on blanks):
#   tests[:pytest args]      the driver's `python -m pytest tests/ -x -q -m gpu`, clean env (e.g. "tests:tests/test_gpu_ranges.py")
#   testsd[:pytest args]     the same, verbose, with per-test timeouts and a parity log
#   testsv:<variant>[:args]  the same against exp/<variant>'s libraries (SHIRLEY_LIB_DIR)
#   smoke                    __graft_entry__.smoke()
#   bench[:bench.py args]    one bench line (default: the driver's defaults)
#   ab:<spec>;<spec>;...     interleaved A/B, one bench line per spec "variant|ENV=V ...|bench flags"
#                            (variant "main" = the in-tree build, else exp/<variant>, see tools/variant.sh);
#                            AB_REPS (default 2) rounds over the specs, AB_STEPS (default 3) steps each
#   prof[:bench.py args]     rocprofv3 --kernel-trace --stats (kernel_stats.csv under <tag>/prof)
#   pmc:<COUNTERS>[:args]    one rocprofv3 --pmc pass (counters comma-separated, one block's limits)
#   py:<script> [args]       a python tool (e.g. "py:tools/shard_balance.py gpurun_out/x/shard.json")
#   sh:<command line>        any command, run by bash -c as written
# Recipes (profiles/<round>/ evidence):
#   kernel stats + HBM traffic:  prof pmc:FETCH_SIZE pmc:WRITE_SIZE, then
#                                python tools/pmc_traffic.py gpurun_out/<tag> profiles/<round> "<workload>" sah
#   VALU issue / lane use:       "pmc:SQ_WAVE_CYCLES,SQ_ACTIVE_INST_VALU,SQ_INSTS_VALU,SQ_THREAD_CYCLES_VALU,
#                                SQ_INSTS_VALU_ADD_F64,SQ_INSTS_VALU_MUL_F64,SQ_INSTS_VALU_FMA_F64,SQ_INSTS_SALU:
#                                --steps 1 --warmup 0 --no-cpu --no-configs", then
#                                python tools/pmc_valu.py profiles/<round> 4 gpurun_out/<tag>/pmc_SQ_WAVE_CYCLES_...
# Examples:
#   gpurun -- 'bash tools/gpu.sh r03a tests smoke "bench:--steps 5" "prof:--steps 3 --no-cpu --no-configs"'
#   gpurun -- 'bash tools/gpu.sh r03b "ab:main||;f32s||;main||;f32s||"'
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp

tag=$1; shift
out=gpurun_out/$tag
mkdir -p "$out"
echo "tools/gpu.sh $tag $*" > "$out/invocation.txt"
git_head=$(cat .git_head 2>/dev/null || true)
[ -n "$git_head" ] && echo "tree $git_head" >> "$out/invocation.txt"
n=0

summary() {  # one line of a bench log: value, kernel time, chunk / passes
  tail -1 "$1" | python3 -c 'import sys,json
d=json.loads(sys.stdin.read()); c=d["config"]; r=d["roofline"]
print(d["value"], "Msamples/s", d["ms_per_step"], "ms/step (device", d.get("device_ms_per_step"), ") trace",
      r["kernel_ms"], "ms x", r.get("launches_per_step"), "chunk", c.get("sample_chunk"), "passes", c.get("sample_passes"))' 2>/dev/null
}

for step in "$@"; do
  n=$((n+1))
  name=${step%%:*}
  args=""
  [ "$name" != "$step" ] && args=${step#*:}
  log="$out/$(printf %02d $n)_$name.log"
  case $name in
    tests)  # the driver's own command (`python -m pytest tests/ -x -q -m gpu`, clean environment);
            # the junit report only records per-test outcomes and times for profiles/<round>/
      env -u SHIRLEY_LIB_DIR -u SHIRLEY_ASSETS -u SHIRLEY_PARITY_LOG timeout -k 10 900 python -m pytest ${args:-tests/} \
        -x -q -m gpu --junitxml="$out/junit_$n.xml" > "$log" 2>&1
      rc=$?; echo "[$n tests] rc=$rc $(tail -1 "$log")" ;;
    testsd)  # diagnostic form: verbose, per-test thread timeouts, parity log
      SHIRLEY_PARITY_LOG=$PWD/$out/parity.jsonl timeout -k 10 900 python -u -m pytest ${args:-tests} -m gpu -x -v \
        --timeout 120 --timeout-method thread -p no:cacheprovider > "$log" 2>&1
      rc=$?; echo "[$n testsd] rc=$rc $(tail -1 "$log")" ;;
    testsv)  # testsv:<variant>[:pytest args] — the GPU tests against exp/<variant>'s libraries
      v=${args%%:*}
      targs=""
      [ "$v" != "$args" ] && targs=${args#*:}
      SHIRLEY_LIB_DIR=$PWD/exp/$v timeout -k 10 900 python -u -m pytest ${targs:-tests} -m gpu -x -v --timeout 120 \
        --timeout-method thread -p no:cacheprovider > "$log" 2>&1
      rc=$?; echo "[$n tests on exp/$v] rc=$rc $(tail -1 "$log")" ;;
    smoke)
      timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > "$log" 2>&1
      rc=$?; echo "[$n smoke] rc=$rc $(tail -1 "$log")" ;;
    bench)
      timeout -k 10 600 python -u bench.py $args > "$log" 2>&1
      rc=$?; echo "[$n bench $args] rc=$rc $(summary "$log")" ;;
    ab)
      IFS=';' read -r -a specs <<< "$args"
      rc=0
      for rep in $(seq 1 ${AB_REPS:-2}); do
        i=0
        for spec in "${specs[@]}"; do
          i=$((i+1))
          IFS='|' read -r v envs flags <<< "$spec"
          if [ "$v" = "main" ]; then dir=""; else dir="$PWD/exp/$v"; fi
          l="$out/$(printf %02d $n)_ab_${rep}_$i.log"
          env SHIRLEY_LIB_DIR=$dir $envs timeout -k 10 400 python bench.py --steps ${AB_STEPS:-3} --warmup 1 --no-cpu \
            --no-configs $flags > "$l" 2>&1
          rc=$?
          echo "[$n ab $rep/$i $spec] rc=$rc $(summary "$l")"
          [ $rc -eq 0 ] || { tail -5 "$l"; break 2; }
        done
      done ;;
    prof)
      timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/prof" -o run -- \
        python3 bench.py ${args:---steps 3 --warmup 1 --no-cpu --no-configs} > "$log" 2>&1
      rc=$?; echo "[$n prof] rc=$rc $(summary "$log")"
      find "$out/prof" -name "*kernel_stats.csv" | head -3 ;;
    pmc)
      counters=${args%%:*}
      pargs=""
      [ "$counters" != "$args" ] && pargs=${args#*:}
      d="$out/pmc_$(echo "$counters" | tr ',' '_')"
      log="$d.log"  # (tools/pmc_valu.py reads the pass's bench line from <pass dir>.log)
      timeout -s KILL 300 rocprofv3 --pmc $(echo "$counters" | tr ',' ' ') --output-format csv -d "$d" -o run -- \
        python3 bench.py ${pargs:---steps 1 --warmup 0 --no-cpu --no-configs} > "$log" 2>&1
      rc=$?; echo "[$n pmc $counters] rc=$rc"
      find "$d" -name "*counter_collection.csv" | head -2 ;;
    sh)  # sh:<command line> — run as written by bash (quoting kept)
      timeout -k 10 600 bash -c "$args" > "$log" 2>&1
      rc=$?; echo "[$n sh $args] rc=$rc"; tail -30 "$log" ;;
    py)
      timeout -k 10 900 python -u $args > "$log" 2>&1
      rc=$?; echo "[$n py $args] rc=$rc"; tail -3 "$log" ;;
    *)
      echo "unknown step $name"; rc=2 ;;
  esac
  if [ $rc -ne 0 ]; then
    echo "step $n ($name) failed rc=$rc: stopping"; tail -20 "$log" 2>/dev/null
    exit $rc
  fi
done
