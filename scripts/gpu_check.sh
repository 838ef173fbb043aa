#!/bin/bash
# GPU-box check: each GPU step under its own timeout; test failures (rc 1) continue, crashes/timeouts stop.
# usage: bash scripts/gpu_check.sh <name> <timeout_s> <cmd...>   (one step)   -- chain steps with &&
set -u
out=gpurun_out; mkdir -p "$out/$(dirname "$1")"
name=$1; t=$2; shift 2
timeout -k 10 "$t" "$@" > "$out/$name.log" 2>&1; rc=$?
echo "== $name rc=$rc"; tail -n 25 "$out/$name.log"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
exit 0
