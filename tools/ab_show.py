"""Summarise gpurun_out/ab/*.log bench lines (tools/ab_run.sh)."""
import glob
import json

for f in sorted(glob.glob('gpurun_out/ab/*_*.log')):
    rows = [x for x in open(f) if x.startswith('{')]
    if not rows:
        print(f, 'no bench line')
        continue
    d = json.loads(rows[-1])
    iso = d['roofline']['isolated']['stage_ms']
    print(f.split('/')[-1], round(d['value']), d['ms_per_step'],
          'iso', {k: round(v, 3) for k, v in iso.items() if v > 0.05})
