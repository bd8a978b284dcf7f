#!/bin/bash
# Round-end set on the final sources: every GPU test + the headline profile
# set (tools/final_session.sh), then the per-rank strong-scaling probe
# (tools/scaling_probe.sh). Usage: tools/final_session3.sh TAG
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
bash tools/final_session.sh $1 || exit 1
bash tools/scaling_probe.sh $1
