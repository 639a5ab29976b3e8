#!/bin/bash
# Local helper (runs in the build container, not on the GPU box): rebuild libreidmi.so from the
# current sources, then send the tree to the GPU box with gpurun.
# usage: tools/run_gpu.sh TIMEOUT 'NAME:SECONDS:CMD' ...   (steps as tools/gpu_suite.sh)
set -e
cd "$(dirname "$0")/.."
python -c "
import sys
sys.path.insert(0, 'multimodal-reid_amd')
import build_lib
build_lib.build(verbose=True)"
t=$1; shift
args=""
for a in "$@"; do args="$args \"$a\""; done
rm -rf gpurun_out/*
set +e
/usr/local/graft/bin/gpurun --timeout "$t" -- "tools/gpu_suite.sh $args"
