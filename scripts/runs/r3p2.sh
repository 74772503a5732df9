# round-3 profiles of the final build: C4 (PARK) and C5 (plain)
cd $GRAFT_REPO_ROOT && \
timeout -k 10 1000 bash scripts/profile.sh r3p_c4 --schedule park --workload c4_bunny4k && \
timeout -k 10 1000 bash scripts/profile.sh r3p_c5 --schedule plain --workload c5_mixed
