#!/bin/bash
# One GPU-box pass of several steps, each under its own time limit.  A step that fails
# ordinarily (a test failure, exit 1) does not stop the pass; a step that aborts, faults or
# times out (exit 124, 134, 137, 139 or a signal) ends it -- nothing more runs on the GPU.
# usage: bash tools/gpu_pass.sh TAG "name|seconds|command" ...
tag=$1; shift
mkdir -p gpurun_out/$tag
for spec in "$@"; do
  name=${spec%%|*}; rest=${spec#*|}; secs=${rest%%|*}; cmd=${rest#*|}
  echo "== $name ($secs s): $cmd" >> gpurun_out/$tag/pass.log
  timeout -k 10 $secs bash -c "$cmd" > gpurun_out/$tag/$name.log 2>&1
  rc=$?
  echo "   rc $rc" >> gpurun_out/$tag/pass.log
  tail -n 3 gpurun_out/$tag/$name.log | cut -c1-300 >> gpurun_out/$tag/pass.log
  case $rc in
    0|1|2|5) ;;
    *) echo "stopping: $name exited $rc" >> gpurun_out/$tag/pass.log; cat gpurun_out/$tag/pass.log; exit $rc ;;
  esac
done
cat gpurun_out/$tag/pass.log
