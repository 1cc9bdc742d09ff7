#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/ab.sh "" w4 w5
