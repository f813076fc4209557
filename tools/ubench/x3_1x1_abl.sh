set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for r in 1 2; do
for a in 0 1 2 8 16 24 32; do
  timeout -k 10 120 ./tools/ubench/x3_1x1_check 65536 $a || exit 1
done; done
