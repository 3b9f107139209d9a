#!/bin/bash
# both round-4 A/B sets in one box: the aggregated binning (gpu_r4_agg3.sh)
# and the persistent blend (gpu_r4_persist.sh)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
bash tools/gpu_r4_agg3.sh && bash tools/gpu_r4_persist.sh
