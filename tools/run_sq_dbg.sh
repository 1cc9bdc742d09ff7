set -o pipefail
export TMPDIR=/tmp
bash tools/pmc_sq.sh sq_c3 || exit 1
bash tools/emit_dbg.sh || exit 1
