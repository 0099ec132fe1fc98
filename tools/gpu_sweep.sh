#!/bin/bash
# Knob sweep (run on the GPU box via gpurun): config-5 stage timings per library variant and env
# setting (tools/gemm_probe.py), then config-2 bench lines per K1m env setting.  Each GPU step is
# time-limited; the chain stops at the first failure.
#   TAG=name  G5_LIBS=a.so,b.so  G5_ENVS="E1 E2"  C2_ENVS="E1 E2"  G5_N=10000000
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-sweep}
mkdir -p $OUT
if [ -n "${G5_ENVS+x}" ]; then
  EARGS=""; for e in ${G5_ENVS}; do EARGS="$EARGS --env $e"; done
  VRQ_LIBS=${G5_LIBS:-} timeout -k 10 ${G5_T:-500} python -u tools/gemm_probe.py --n ${G5_N:-10000000} --iters 3 ${G5_ARGS:-} $EARGS > $OUT/g5.jsonl 2> $OUT/g5.err || { echo G5_FAIL; tail -20 $OUT/g5.err; exit 1; }
  cat $OUT/g5.jsonl
fi
for e in ${C2_ENVS:-}; do
  f=$OUT/c2_${e//\//_}
  env $(echo $e | tr ',' ' ') timeout -k 10 200 python -u bench.py --config ${C2_CFG:-c2} --no-cpu-baseline --no-recall --no-encode --steps 20 --warmup 3 > $f.json 2> $f.err || { echo C2_FAIL $e; tail -20 $f.err; exit 1; }
  python -c "import json;d=json.load(open('$f.json'));print('$e', round(d['ms_per_step'],4), {k:round(v,4) for k,v in d['phase_ms'].items()}, round(d['roofline']['frac'],3))"
done
echo done
