set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/s2
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/s2/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -30 gpurun_out/s2/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/s2/pytest_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s2/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -20 gpurun_out/s2/smoke.log; exit 1; }
tail -1 gpurun_out/s2/smoke.log
timeout -k 10 300 python bench.py > gpurun_out/s2/bench.json 2> gpurun_out/s2/bench.err || { echo BENCH_FAIL; tail -20 gpurun_out/s2/bench.err; exit 1; }
cat gpurun_out/s2/bench.json
