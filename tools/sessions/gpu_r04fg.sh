#!/bin/bash
# Round 4, sessions f + g in one call: the variant A/B (gpu_r04f.sh) and the knock-out PMC
# passes (gpu_r04g.sh).
# Usage: bash tools/sessions/gpu_r04fg.sh TAG
set -o pipefail
TAG=${1:-r04fg}
bash tools/sessions/gpu_r04g.sh ${TAG}_g || exit 1
bash tools/sessions/gpu_r04f.sh ${TAG}_f || exit 1
