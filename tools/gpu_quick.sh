#!/bin/bash
# GPU tests (optionally a -k filter in $1) + per-op breakdown bench
set -o pipefail
K=${1:-}
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${K:+-k "$K"} > gpurun_out/gpu_tests.log 2>&1 || { echo "[quick] tests rc=$?"; tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 --kernel-breakdown > gpurun_out/bench_kb.json 2> gpurun_out/breakdown.txt || { echo "[quick] kb rc=$?"; tail -20 gpurun_out/breakdown.txt; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/bench_kb.json'));print('value',d['value'],'ms',d['ms_per_step'])"
echo "[quick] ok"
