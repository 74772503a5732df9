# round-3 profiles of the final build: kernel trace + PMC passes (scripts/profile.sh) for C3 (PARK), C3 adaptive,
# C2 (plain)
cd $GRAFT_REPO_ROOT && \
timeout -k 10 900 bash scripts/profile.sh r3p_c3 --schedule park && \
timeout -k 10 900 bash scripts/profile.sh r3p_c3a --schedule park --adaptive && \
timeout -k 10 900 bash scripts/profile.sh r3p_c2 --schedule plain --workload c2_final
