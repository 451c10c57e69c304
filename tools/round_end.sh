#!/bin/bash
# The end-of-round evidence in one GPU call: tools/round_end.sh TAG
#   1. tools/profile.sh TAG: rocprofv3 kernel trace of the default bench and
#      the separate --pmc passes (FETCH_SIZE, WRITE_SIZE, SQ counters);
#   2. profiles/pmc_traffic.json rebuilt from those passes (bench.py reads it
#      for roofline.traffic), also kept as gpurun_out/prof_TAG/pmc_traffic.json;
#   3. tools/final_round.sh TAG: every bench line, now carrying that traffic.
set -euo pipefail
TAG=${1:-r05}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
bash tools/profile.sh "$TAG"
python3 tools/make_traffic.py "gpurun_out/prof_$TAG" > "gpurun_out/prof_$TAG/pmc_traffic.json"
cp "gpurun_out/prof_$TAG/pmc_traffic.json" profiles/pmc_traffic.json
bash tools/final_round.sh "$TAG"
