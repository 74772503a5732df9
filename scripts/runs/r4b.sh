# round-3 final adaptive schedule: rocprofv3 kernel trace + PMC passes of C3 adaptive (PARK), then the N>1
# bench path rehearsed with 2 ranks on one GPU (gloo barrier, C4 at 32 spp)
cd $GRAFT_REPO_ROOT && \
timeout -k 10 1000 bash scripts/profile.sh r4b_c3a --schedule park --adaptive && \
NPROC=2 timeout -k 10 450 bash scripts/multirank_rehearsal.sh --spp 32
