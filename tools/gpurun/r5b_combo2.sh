#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/gpurun/r5b_km_ab.sh && bash tools/gpurun/r5b_stored_prof.sh
