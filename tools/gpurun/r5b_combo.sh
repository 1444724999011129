#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/gpurun/r5b_gb.sh && bash tools/gpurun/r5b_stored.sh && bash tools/gpurun/r5b_km_pmc.sh
