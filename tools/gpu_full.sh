#!/bin/bash
# GPU tests + default bench + per-op breakdown, each step under its own time limit
set -o pipefail
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo "[full] tests rc=$?"; tail -20 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 200 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "[full] bench rc=$?"; exit 1; }
cat gpurun_out/bench.json
timeout -k 10 200 python bench.py --no-cpu-baseline --steps 10 --kernel-breakdown > gpurun_out/bench_kb.json 2> gpurun_out/breakdown.txt || { echo "[full] kb rc=$?"; exit 1; }
echo "[full] ok"
