# tests/asan/host_asan under a torch-initialised parent (tools/asan_parent_probe.py),
# three runs with the small-burst forms on (default) and three with them off
# (NET2_BURST_WAVE_MAX=0); PROBE_ASAN_OPTIONS sets the ASan options (e.g.
# detect_leaks=0), 75 s a run.
set -u
mkdir -p gpurun_out
for k in 1 2 3; do
  for mode in on off; do
    if [ $mode = off ]; then export NET2_BURST_WAVE_MAX=0; else unset NET2_BURST_WAVE_MAX; fi
    timeout -k 10 75 python3 tools/asan_parent_probe.py torch gpurun_out/hang_${mode}_$k.txt > gpurun_out/hang_${mode}_$k.log 2>&1
    echo "$mode $k rc=$?" >> gpurun_out/hang_summary.txt
  done
done
exit 0
