#!/bin/bash
# GPU A/B of the partial-view (or full-view) tick kernel between this tree and another
# checkout of the repo (e.g. a git worktree of an earlier commit, built in place), interleaved:
#   bash scripts/ab_trees.sh <tag> <other-tree-dir> [reps] [pview|full]
set -euo pipefail
: "${GRAFT_REPO_ROOT:?run on the GPU box (gpurun exports GRAFT_REPO_ROOT)}"
TAG=$1; OTHER=$2; REPS=${3:-3}; WHAT=${4:-pview}
OUT="$GRAFT_REPO_ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
export TMPDIR=/tmp
for i in $(seq "$REPS"); do
    for side in new old; do
        dir="$GRAFT_REPO_ROOT"; [ "$side" = old ] && dir="$GRAFT_REPO_ROOT/$OTHER"
        if [ "$WHAT" = full ]; then
            (cd "$dir" && timeout -k 10 150 python3 -u bench.py --steps 20 --warmup 5 \
                --no-cpu-baseline --no-pview) > "$OUT/$side.$i.log" 2>&1
        else
            (cd "$dir" && timeout -k 10 150 python3 -u scripts/bench_pview.py --steps 10 --warmup 5 \
                --no-cpu-baseline) > "$OUT/$side.$i.log" 2>&1
        fi
        echo "$side $i $(tail -1 "$OUT/$side.$i.log" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("kernel_ms=%.3f" % d["roofline"]["kernel_ms_per_tick"])')"
    done
done
