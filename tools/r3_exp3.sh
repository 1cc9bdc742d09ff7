#!/bin/bash
# count pass rows per wave (byte-domain med: the row above costs only its bytes)
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/ab.sh "" gbm gr1 gr2
