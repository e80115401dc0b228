# look-back embed phase stamps at the headline shape (first 4096 slots: group 0's chunks 0..127),
# with and without the finished-flag recheck
cd "$GRAFT_REPO_ROOT" || exit 9
for rc in 0 1; do
  echo "== CODEC_PEE_1P_RECHECK=$rc"
  CODEC_PEE_1P_RECHECK=$rc timeout -k 10 200 python tools/lb_trace.py run 256 2>&1 | grep -v amdgpu.ids || exit 1
done
