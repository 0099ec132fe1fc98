#!/bin/bash
# K1m thresholded pass alone (tools/probes/mfma_bisect_<bits>, random codes, nq = 1024) at the config-2
# size with no hits (tau 0), ~3 and ~160 hits per query (tau 440 / 458), and at 10M rows: locates the
# fixed cost above the MFMA time at 1M rows.  Each run is time-limited; the chain stops at a failure.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/${TAG:-c2b}
for b in ${BITS:-0 1 2 4}; do for n in 1000000 10000000; do for tau in 0 440 458; do
  timeout -k 10 60 ./tools/probes/mfma_bisect_$b $n 1024 $tau | sed "s/^/{\"tau\": $tau, \"r\": /; s/$/}/" >> gpurun_out/${TAG:-c2b}/r.jsonl || exit 1
done; done; done
cat gpurun_out/${TAG:-c2b}/r.jsonl
