#!/bin/bash
# rocprofv3 PMC passes with caller-chosen counter groups (csv); run on the GPU box.
#   tools/pmc_groups.sh <outdir> "<group1 counters>" ["<group2>" ...] -- <python script> [args...]
out="$1"; shift
groups=()
while [ "$#" -gt 0 ] && [ "$1" != "--" ]; do groups+=("$1"); shift; done
shift
root="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
script="$1"; shift
mkdir -p "$root/$out"; cd /tmp && export TMPDIR=/tmp
set -e
i=0
for g in "${groups[@]}"; do
  i=$((i + 1))
  # shellcheck disable=SC2086
  timeout -k 10 100 rocprofv3 --pmc $g --output-format csv -d "$root/$out/g$i" -o run -- python3 "$root/$script" "$@"
done
