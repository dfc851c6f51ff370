#!/bin/bash
# pipe A/B, then the grouped-walk defaults + tests
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash scripts/r06_pipe.sh && bash scripts/r06_group3.sh
