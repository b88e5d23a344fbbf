#!/bin/bash
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r06b; mkdir -p $OUT
timeout -k 10 200 python -u scripts/debug/drain_rowdiff.py > $OUT/diff_h0.log 2>&1; cat $OUT/diff_h0.log | tail -20
GSP_TEST_PV_DRAIN_LDS=300 timeout -k 10 200 python -u scripts/debug/drain_rowdiff.py > $OUT/diff_hub.log 2>&1; tail -20 $OUT/diff_hub.log
