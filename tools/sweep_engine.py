"""A/B the engine's scheduling knobs on the bench workload.
Usage: python tools/sweep_engine.py 'LANE0_CU_SHARE=0.5' 'LANE0_CU_SHARE=0.625' 'Plan.MULTI_STREAM=0' ...
Each argument is one configuration of DBSREngine (or Plan.*) class attributes; prints bursts/s per configuration."""
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)

CHILD = r'''
import sys, runpy
sys.argv = ['bench.py', '--steps', '30', '--warmup', '5', '--no-cpu-baseline']
import dbsr_amd.engine as e
for kv in %r.split(','):
    if kv:
        k, v = kv.split('=')
        cls = e.Plan if k.startswith('Plan.') else e.DBSREngine
        k = k.split('.')[-1]
        setattr(cls, k, type(getattr(cls, k))(float(v)) if '.' in v else int(v))
runpy.run_path('bench.py', run_name='__main__')
'''

for cfg in sys.argv[1:]:
    out = subprocess.run([sys.executable, '-c', CHILD % cfg], cwd=REPO, capture_output=True, text=True, timeout=300)
    line = [ln for ln in out.stdout.splitlines() if ln.startswith('{')]
    if not line:
        print(cfg, 'FAILED', out.stderr[-500:])
        sys.exit(1)
    d = json.loads(line[-1])
    print('%-45s %8.1f bursts/s %7.3f ms' % (cfg, d['value'], d['ms_per_step']), flush=True)
