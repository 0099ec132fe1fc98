set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pr
VRQ_LIB=tools/probes/g5/lib_p1.so timeout -k 10 600 python -u -m pytest tests/test_gpu_mfma.py tests/test_gpu_fullsize.py tests/test_gpu_parity.py tests/test_gpu_scale.py tests/test_gpu_dist.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pr/pytest_p1.log 2>&1 || { echo P1_TEST_FAIL; tail -40 gpurun_out/pr/pytest_p1.log; exit 1; }
tail -2 gpurun_out/pr/pytest_p1.log
TAG=pr TESTS=0 VARIANTS="p0c2=tools/probes/g5/lib_p0.so:c2 p1c2=tools/probes/g5/lib_p1.so:c2 p0c4=tools/probes/g5/lib_p0.so:c4 p1c4=tools/probes/g5/lib_p1.so:c4" BENCH_T=300 bash tools/gpu_r3.sh || exit 1
RUNS="c5:1024" TAG=pr5 PMC=1 bash tools/prof_r3.sh
