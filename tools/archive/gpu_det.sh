#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT}"
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -q -rf --timeout 120 --timeout-method thread -k "deterministic or lg_proj" 2>&1 | tail -5
