#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash scripts/r06_env_abn.sh && bash scripts/r06_attn_diag.sh
