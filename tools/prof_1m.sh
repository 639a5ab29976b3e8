#!/bin/bash
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_1m -o rr -- \
  python tools/scale_vitl_1m.py --no-embed > gpurun_out/rr1m_under_rocprof.json
