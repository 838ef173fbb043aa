#!/bin/bash
# Same-box A/B of (library, env) arms on one bench workload:
#   bash scripts/ab_arms.sh <tag> "<bench args>" <arm>...     arm = <lib.so or "-">[,VAR=value...]
# e.g. bash scripts/ab_arms.sh ca64 "--workload humanoid_ca" lib/ab/lib_head.so - -,MPPI_FC_WIDE=1
set -u
tag=$1; args=$2; shift 2
mkdir -p gpurun_out
i=0
for arm in "$@"; do
  i=$((i + 1))
  IFS=, read -r lib envs <<< "$arm"
  envv=()
  [ "$lib" != "-" ] && envv+=("MPPI_HIP_LIB=$lib")
  if [ -n "${envs:-}" ]; then IFS=, read -ra extra <<< "$envs"; envv+=("${extra[@]}"); fi
  log=gpurun_out/ab_${tag}_$i.log
  env "${envv[@]}" timeout -k 10 200 python3 bench.py $args --no-cpu-baseline --no-traffic --no-kernel-trace > $log 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "== $tag arm $arm rc=$rc"; tail -5 $log; exit $rc; fi
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(f\"{sys.argv[2]:>8} {sys.argv[3]:<40} value {d['value']:.4g} ms/step {d['ms_per_step']:.4f} rollout {r['avg_launch_us']:.1f} us frac {r['frac']:.4f}\")" $log $tag "$arm"
done
