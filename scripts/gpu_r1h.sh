#!/bin/bash
# Wide x3b (8-wave, LDS b1 / w2) as default: GPU suite + smoke + default bench + profile, then config 5.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
scripts/gpu_final.sh prof_r1h && scripts/gpu_cfg5_ab.sh base
