# round-3 final adaptive build: rocprofv3 kernel trace + PMC passes of C3 adaptive (PARK)
cd $GRAFT_REPO_ROOT && timeout -k 10 1000 bash scripts/profile.sh r4e_c3a --schedule park --adaptive
