#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/ab.sh "" base2 rol5 rol4
bash tools/ab.sh "--workload c4" base2 rol5
