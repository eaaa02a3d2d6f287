ST=$GRAFT_REPO_ROOT/gpurun_out/sb_states.bin
for b in ${SB:-w3 w4}; do echo -n "$b "; timeout -k 10 60 tools/_bin/stencil_bench_$b $ST || exit $?; done
