# round-3: r4c (adaptive pixel order A/B + adaptive tests), then the 2-rank rehearsal of bench.py's N>1 path
cd $GRAFT_REPO_ROOT && timeout -k 10 900 bash scripts/r4c.sh && NPROC=2 timeout -k 10 450 bash scripts/multirank_rehearsal.sh --spp 32
