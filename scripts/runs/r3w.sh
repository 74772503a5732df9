# round-3 re-entry: the r3u check (GPU tests, smoke, default bench lines, offset A/B) then the r3v adaptive tuning A/B
cd $GRAFT_REPO_ROOT && timeout -k 10 1000 bash scripts/r3u.sh && timeout -k 10 900 bash scripts/r3v.sh
