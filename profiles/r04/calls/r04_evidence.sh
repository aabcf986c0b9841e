#!/bin/bash
cd ${GRAFT_REPO_ROOT:-.}
bash scripts/round_evidence.sh r04
