#!/bin/bash
# late round 3: encode variants A/B, then the snappy next-chunk prefetch A/B
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/rounds/gpu_enc_persist.sh || exit 1
bash tools/rounds/gpu_snap_pf.sh || exit 2
