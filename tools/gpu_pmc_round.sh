cd "${GRAFT_REPO_ROOT:-/root/repo}"
PMC_SIZES="4096 262144" bash tools/gpu_pmc.sh && bash tools/gpu_rigid_probe.sh r02c
