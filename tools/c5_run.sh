set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/${TAG:-c5a}
timeout -k 10 300 python -u -m pytest tests/test_gpu_gemm.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG:-c5a}/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -30 gpurun_out/${TAG:-c5a}/pytest.log; exit 1; }
tail -1 gpurun_out/${TAG:-c5a}/pytest.log
timeout -k 10 400 python bench.py --config c5 --steps 3 --warmup 1 --no-recall > gpurun_out/${TAG:-c5a}/bench.json 2> gpurun_out/${TAG:-c5a}/bench.err || { echo BENCH_FAIL; tail -20 gpurun_out/${TAG:-c5a}/bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/${TAG:-c5a}/bench.json'));print('QPS',round(d['value']),{k:round(v,3) for k,v in d['phase_ms'].items()},d['roofline']['frac'],d['roofline_binary']['frac'],d.get('cpu_baseline'))"
