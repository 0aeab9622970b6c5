#!/bin/bash
# A/B of library builds x environment x bench flags.  Each argument: "variant;ENV=V ...;bench flags"
# (variant "main" = the in-tree build, else exp/<variant>).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export SHIRLEY_ASSETS=${SHIRLEY_ASSETS:-$PWD/shirley-raytracing-rs_amd/assets}  # exp/<variant> libs resolve assets here
i=0
for spec in "$@"; do
  i=$((i+1))
  IFS=';' read -r v envs flags <<< "$spec"
  if [ "$v" = "main" ]; then dir=""; else dir="$PWD/exp/$v"; fi
  env SHIRLEY_LIB_DIR=$dir $envs timeout -k 10 300 python bench.py --steps ${AB_STEPS:-3} --warmup 1 --no-cpu --no-configs $flags > gpurun_out/ab2_$i.log 2>&1
  rc=$?
  echo "[$spec] rc=$rc $(tail -1 gpurun_out/ab2_$i.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); c=d["config"]; print(d["value"], "Msamples/s", d["roofline"]["kernel_ms"], "ms", c.get("engine"), c.get("kernel_ms_split"))' 2>/dev/null)"
  [ $rc -eq 0 ] || { tail -3 gpurun_out/ab2_$i.log; exit $rc; }
done
