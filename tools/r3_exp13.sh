#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/ab.sh "" occ8 occ3 occ2 gm2
bash tools/ab.sh "--workload c4" occ8 occ3 gm2
