# look-back embed phase stamps at the headline shape (first 4096 slots: group 0's chunks 0..127)
cd "$GRAFT_REPO_ROOT" || exit 9
timeout -k 10 200 python tools/lb_trace.py run 256 2>&1 | grep -v amdgpu.ids
