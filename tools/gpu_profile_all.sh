#!/bin/bash
# The round's committed profiles in one GPU call: kernel trace + stats, HBM
# counters (FETCH_SIZE / WRITE_SIZE passes) and SQ instruction counters, all
# of the same bench command.  Then: python tools/pmc_to_profile.py <tag>
# usage: tools/gpu_profile_all.sh <tag> [bench args...]
cd "$GRAFT_REPO_ROOT" || exit 1
tag=$1; shift
tools/gpu_prof.sh $tag "$@" > /dev/null && \
tools/gpu_pmc.sh $tag "$@" && \
PMC_GROUPS="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY;SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
  tools/gpu_pmc_sq.sh $tag "$@"
