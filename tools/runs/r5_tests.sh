#!/bin/bash
# Round-5 GPU test pass: the new list/instance tests first, then the whole -m gpu suite.
# Each pytest run is time-limited; a heartbeat file shows progress during long single tests.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-r5t}
mkdir -p $OUT
(while true; do date +%T >> $OUT/heartbeat; sleep 20; done) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
rc=0
timeout -k 10 ${T1:-900} python -u -m pytest ${FIRST:-tests/test_gpu_lists.py} -m gpu -v --maxfail=4 --timeout 400 \
  --timeout-method thread -p no:cacheprovider > $OUT/first.log 2>&1 || rc=$?
tail -5 $OUT/first.log
if [ "$rc" = "0" ] && [ "${ALL:-1}" = "1" ]; then
  timeout -k 10 ${T2:-1200} python -u -m pytest tests -m gpu -v --maxfail=4 --timeout 400 --timeout-method thread \
    -p no:cacheprovider ${DESELECT:-} > $OUT/all.log 2>&1 || rc=$?
  tail -5 $OUT/all.log
fi
exit $rc
