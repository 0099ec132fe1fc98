cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/ab1
for b in 0 0_a5 0_a6 1 8 16 24 0; do for tau in 440 465; do
 timeout -k 10 60 ./tools/probes/mfma_bisect_$b 10000000 1024 $tau | sed "s/^/$b /" >> gpurun_out/ab1/r.txt || exit 1
done; done
cat gpurun_out/ab1/r.txt
