#!/bin/bash
# Usage: bash tools_gpu_check.sh <step-name> <timeout-s> <cmd...>   (used inside gpurun calls)
# Runs one GPU step under its own time limit; exits non-zero (stopping the && chain) on a fault,
# abort, segfault or timeout, but lets ordinary test failures (exit 1) continue to the next step.
name=$1; lim=$2; shift 2
mkdir -p gpurun_out
timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
rc=$?
echo "[$name] exit $rc" | tee -a gpurun_out/steps.log
case $rc in 0|1|2|5) exit 0;; *) exit $rc;; esac
