set -o pipefail
# kernel iteration pass: MFMA-scan parity tests, bisect timings, a short c4 bench
mkdir -p gpurun_out/k
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_mfma.py tests/test_gpu_parity.py} -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/k/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/k/pytest.log; exit 1; }
tail -1 gpurun_out/k/pytest.log
for b in ${BIS:-0 1 2 3}; do for n in ${NS:-100000000}; do timeout -k 5 60 ./tools/probes/mfma_bisect_$b $n 1024 440 || exit 1; done; done
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-recall --no-encode ${BARGS:-} > gpurun_out/k/c4.json 2> gpurun_out/k/c4.err || { tail -20 gpurun_out/k/c4.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/k/c4.json'));print('c4', round(d['value']), round(d['ms_per_step'],2), {k:round(v,3) for k,v in d['phase_ms'].items()}, round(d['roofline']['frac'],3))"
