cd ${GRAFT_REPO_ROOT:-.}
scripts/gpu_steps.sh \
 "pytest_gpu|420|python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread" \
 "hb|300|scripts/ab_host_boundary.sh 'main g1 g2 g8 g4p g2p' c3 1 300" \
 "ab|400|scripts/ab_bench.sh 'base main' 'c3 c5 c2' 2"
