#!/bin/bash
# One GPU session, steps chosen by name (replaces the per-session drivers of earlier rounds).
# Every GPU step has its own time limit; the first timeout, abort or crash ends the script (test
# failures, rc 1, do not). Output: gpurun_out/<tag>/.
# Usage: gpurun --timeout 1200 -- 'bash scripts/gpu_run.sh <tag> <step>...'
#   tests          the GPU suite (pytest -m gpu)
#   tests:<expr>   the GPU tests matching a -k expression
#   smoke          __graft_entry__.smoke()
#   bench          the default bench line (C2 + c4/c5 sub-lines + CPU legs + Node path)
#   quick          the default bench line without CPU legs and the Node path
#   prof           rocprofv3 --kernel-trace --stats of a quick C2 + C4 + C5 run (no CPU legs)
#   prof:<w>[:tag] the same for workload w's line alone (c2, c4, c5: its kernels' averages are per launch)
#   pmc:<w>        FETCH_SIZE / WRITE_SIZE / SQ passes of workload w (c2, c4, c5) (scripts/gpu_pmc.sh)
#   ab:<variant>   quick C2 + C5 lines with exp/<variant>/libdrp.so (scripts/build_variant.sh)
#   probe:<script> python3 scripts/<script> (a measurement script)
#   bin:<path>     a prebuilt measurement binary (e.g. exp/probe_bw from scripts/probe_bw.hip)
#   pack           summarise this session's prof / pmc outputs (kernel_phases.txt, pmc_<w>.json) and
#                  delete their per-dispatch CSVs (gpurun copies back at most 64 MiB)
#   env:K=V        export K=V for the steps that follow (unenv:K unsets it)
#   c2 / c4 / c5   that workload's line alone (no sub-lines, no CPU legs), appended to <step>.log
set -e
export TMPDIR=/tmp
TAG=$1
shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
for step in "$@"; do
  case $step in
    tests | tests:*)
      K=${step#tests}
      K=${K#:}
      set +e
      timeout -k 10 900 python -u -m pytest tests -m gpu ${K:+-k "$K"} --maxfail=8 -v -rA --timeout 150 \
        --timeout-method thread > $OUT/gpu_tests.log 2>&1
      rc=$?
      set -e
      echo "tests rc=$rc: $(tail -1 $OUT/gpu_tests.log)"
      if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
      ;;
    smoke)
      timeout -k 10 150 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
      echo "smoke: $(tail -1 $OUT/smoke.log)"
      ;;
    bench)
      timeout -k 10 600 python -u bench.py > $OUT/bench.log 2>&1
      echo bench done
      ;;
    quick)
      timeout -k 10 300 python -u bench.py --no-cpu > $OUT/bench_quick.log 2>&1
      echo quick done
      ;;
    prof)
      (cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/$OUT/prof -o run -- \
        python3 -u $ROOT/bench.py --steps 5 --warmup 2 --no-cpu > $ROOT/$OUT/bench_prof.log 2>&1)
      echo prof done
      ;;
    prof:*)
      W=${step#prof:}
      T=${W#*:}
      [ "$T" = "$W" ] && T="" || W=${W%%:*}
      (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/$OUT/prof_$W$T -o run -- \
        python3 -u $ROOT/bench.py --workload $W --steps 10 --warmup 2 --no-cpu --no-sub > $ROOT/$OUT/bench_prof_$W$T.log 2>&1)
      echo "prof $W$T done: $(python3 scripts/kstats.py $OUT/prof_$W$T/run_kernel_stats.csv 3 | tr -s ' ' | tr '\n' ';')"
      ;;
    pmc:*)
      W=${step#pmc:}
      F=100000000
      timeout -k 10 700 bash scripts/gpu_pmc.sh $F $W $OUT/pmc_$W
      echo "pmc $W done"
      ;;
    ab:*)
      V=${step#ab:}
      DRP_LIB=exp/$V/libdrp.so timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu \
        > $OUT/ab_$V.log 2>&1
      echo "ab $V done"
      ;;
    probe:*)
      S=${step#probe:}
      timeout -k 10 400 python3 -u scripts/$S > $OUT/probe_${S%%.*}.log 2>&1
      echo "probe $S done"
      ;;
    bin:*)
      B=${step#bin:}
      timeout -k 10 300 ./$B > $OUT/bin_$(basename $B).log 2>&1
      echo "bin $B: $(tr '\n' ';' < $OUT/bin_$(basename $B).log | cut -c1-600)"
      ;;
    pack)
      for d in $OUT/pmc_*/; do
        [ -d "$d" ] || continue
        w=$(basename $d)
        w=${w#pmc_}
        python3 scripts/pmc_kernels.py --dir $d --workload $w $([ $w = c3 ] && echo --calls 2) --write $OUT/pmc_$w.json \
          > $OUT/pmc_$w.txt 2>&1 || true
      done
      T=($OUT/prof/*kernel_trace.csv)
      if [ -f "${T[0]}" ]; then python3 scripts/trace_phases.py ${T[0]} 7 > $OUT/kernel_phases.txt 2>&1 || true; fi
      find $OUT -name "*.csv" ! -name "*kernel_stats.csv" -delete
      echo pack done
      ;;
    env:*)
      export "${step#env:}"
      ;;
    unenv:*)
      unset "${step#unenv:}"
      ;;
    c2 | c3 | c4 | c5)
      timeout -k 10 300 python -u bench.py --workload $step --no-cpu --no-sub --steps 10 --warmup 2 >> $OUT/$step.log 2>&1
      echo "$step (${DRP_CLAIMS:-auto} ${DRP_LIB:-}): $(tail -1 $OUT/$step.log | cut -c1-400)"
      ;;
    *)
      echo "unknown step $step"
      exit 2
      ;;
  esac
done
