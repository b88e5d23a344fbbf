#!/bin/bash
# round 6: config 4 (262,144 nodes, 32 column tiles) with the tables in physically contiguous
# memory (GSP_TEST_SCALE_CONTIG=1) against hipMalloc: timing A/B, then one translation-counter
# pass per variant (the round-4 r04d counters)
cd "$GRAFT_REPO_ROOT" || exit 2
OUT="$GRAFT_REPO_ROOT/gpurun_out/${TAG:-r06c4}"; mkdir -p "$OUT"
export AB_N=262144 AB_G=32 AB_W=2 AB_S=8 AB_TIMEOUT=300
timeout -k 10 900 python3 -u scripts/ab_scale_tiles.py 2 base: contig:GSP_TEST_SCALE_CONTIG=1 > "$OUT/ab.txt" 2>&1 || exit 1
cat "$OUT/ab.txt"
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp || exit 2
for v in 0 1; do
  GSP_TEST_SCALE_CONTIG=$v timeout -k 10 300 rocprofv3 --pmc TCP_UTCL1_REQUEST_sum TCP_UTCL1_TRANSLATION_MISS_sum GRBM_UTCL2_BUSY GRBM_GUI_ACTIVE \
      -d "$OUT/pmc_contig$v" -o run --output-format csv -- python3 "$R/scripts/scale_once.py" > "$OUT/pmc_contig$v.log" 2>&1 || exit $?
  echo "pmc contig=$v done"
done
