#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/ab.sh "--workload c4" k16 k4 k8
