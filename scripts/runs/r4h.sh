# round-3 final build: rocprofv3 kernel trace + PMC passes of C3 (PARK, the bench default), C3 adaptive and C2
cd $GRAFT_REPO_ROOT && \
timeout -k 10 700 bash scripts/profile.sh r4h_c3 --schedule park && \
timeout -k 10 700 bash scripts/profile.sh r4h_c3a --schedule park --adaptive && \
timeout -k 10 700 bash scripts/profile.sh r4h_c2 --schedule plain --workload c2_final
