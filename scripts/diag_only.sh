cd $GRAFT_REPO_ROOT
for v in 1e4 1e7; do DIAG_V=$v timeout -k 10 120 python scripts/diag_stamps.py 2>&1 | grep -v amdgpu.ids || exit 3; done
