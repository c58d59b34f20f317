# End-of-round measurements against one kernel build, in GPU calls of a few
# minutes each (STAGE):
#   profile  rocprofv3 kernel trace + PMC passes per config (PCFGS), folded
#            into profiles/pmc_<cfg>.json and profiles/$ROUND/kernel_stats_*
#            (tools/gpu_profile_round.sh);
#   bench    the default bench line (what the driver runs), then every
#            config's own line (tools/gpu_bench_all.sh; SKIP_PYTEST=1 to
#            leave the GPU tests out) -- after `profile`, so every line joins
#            the counters of its own build.
# Outputs under gpurun_out/; copy what is kept into profiles/$ROUND/.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
export ROUND=${ROUND:-round5}
case ${STAGE:-bench} in
profile)
  bash tools/gpu_profile_round.sh ;;
bench)
  timeout -k 10 600 python bench.py > gpurun_out/bench_default.log 2>&1
  rc=$?; echo "bench default rc=$rc"; tail -1 gpurun_out/bench_default.log | cut -c1-300
  [ $rc -ne 0 ] && exit $rc
  bash tools/gpu_bench_all.sh ;;
trace_default)
  # the driver's own command under the kernel tracer: its dominant kernel's
  # trace average against the line's HIP-event kernel time
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_default -o run --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_default_traced.log 2>&1
  rc=$?; echo "trace default rc=$rc"; [ $rc -ne 0 ] && exit $rc
  python3 tools/default_trace_summary.py gpurun_out/prof_default/run_kernel_stats.csv gpurun_out/bench_default_traced.log gpurun_out/prof_default/run_kernel_trace.csv > gpurun_out/default_cmd_trace_summary.json &&
  cp gpurun_out/prof_default/run_kernel_stats.csv gpurun_out/kernel_stats_default_cmd.csv &&
  rm -f gpurun_out/prof_default/run_kernel_trace.csv && cat gpurun_out/default_cmd_trace_summary.json ;;
*)
  echo "STAGE=profile|bench|trace_default" >&2; exit 2 ;;
esac
