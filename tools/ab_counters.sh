#!/bin/bash
# Counter passes for an A/B of library builds (run on the GPU box via gpurun): for each library in LIBS
# and the one CMD (its {lib} replaced by the library path), a kernel-trace pass (per-dispatch durations)
# and three --pmc passes of their own (MI355X_MICROARCH.md: one run per counter set, never combined
# with a trace domain):
#   clk: GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES   (clock, MFMA busy)
#   sq:  SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA
#        SQ_INSTS_VALU SQ_INSTS_SALU                                               (where wave time goes)
#   lds: SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_UNALIGNED_STALL
#        SQ_BUSY_CYCLES                                                            (LDS pressure)
# tools/ab_counters.py condenses them into one JSON line per (library, kernel).
#   TAG=name LIBS="a.so b.so" CMD="python3 tools/stage_bench.py --libs {lib} --cases 1000000:1024 --reps 3 --rounds 1"
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-ab}
mkdir -p $OUT
i=0
for lib in $LIBS; do
  i=$((i + 1))
  D=$OUT/lib$i
  mkdir -p $D
  echo "$lib" > $D/lib.txt
  C=${CMD//\{lib\}/$lib}
  timeout -k 10 ${PT:-300} rocprofv3 --kernel-trace --output-format csv -d $D/trace -o run -- $C > $D/trace.log 2>&1 || { echo TRACE_FAIL $lib; tail -20 $D/trace.log; exit 1; }
  timeout -k 10 ${PT:-300} rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES -d $D/clk -o run --output-format csv -- $C > $D/clk.log 2>&1 || { echo CLK_FAIL $lib; tail -20 $D/clk.log; exit 1; }
  timeout -k 10 ${PT:-300} rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_SALU -d $D/sq -o run --output-format csv -- $C > $D/sq.log 2>&1 || { echo SQ_FAIL $lib; tail -20 $D/sq.log; exit 1; }
  timeout -k 10 ${PT:-300} rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_UNALIGNED_STALL SQ_BUSY_CYCLES -d $D/lds -o run --output-format csv -- $C > $D/lds.log 2>&1 || { echo LDS_FAIL $lib; tail -20 $D/lds.log; exit 1; }
  echo "== $lib done"
done
python3 tools/ab_counters.py $OUT > $OUT/ab_counters.jsonl && cat $OUT/ab_counters.jsonl
# keep the condensed lines only
rm -rf $OUT/lib*/trace $OUT/lib*/clk $OUT/lib*/sq $OUT/lib*/lds
