# A/B of the stream-priority schedule (SDREAMER_PRIO): bench (no probes) twice each, alternating, then the timeline
set -e
for i in 1 2; do
  for P in 0 1; do
    SDREAMER_PRIO=$P timeout -k 10 200 python bench.py --no-roofline --no-cpu-baseline --steps 30 > gpurun_out/r03e_prio${P}_$i.json 2>/dev/null
  done
done
SDREAMER_PRIO=1 timeout -k 10 200 python tools/timeline.py 8 > gpurun_out/r03e_timeline_prio1.txt 2>&1
