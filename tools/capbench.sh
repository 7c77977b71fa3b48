for c in ${CAPS:-0.25 0.375 0.5}; do
  timeout -k 10 200 python3 -c "
import sys, runpy
sys.argv = ['bench.py', '--steps', '20', '--warmup', '5', '--no-cpu-baseline']
import dbsr_amd.engine as e
e.DBSREngine.LANE0_CU_SHARE = $c
runpy.run_path('bench.py', run_name='__main__')
" 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$c', d['value'], d['ms_per_step'])" || exit 1
done
