#!/bin/bash
# Round 4, call 22: round-end evidence on the library with the persistent bounce grid at 75 %.
cd ${GRAFT_REPO_ROOT:-.}
bash scripts/round_evidence.sh r04
