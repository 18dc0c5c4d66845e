#!/bin/bash
# r04n: Process-API fast paths -- engine / registry / invoke GPU tests, then the loop profile.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r04n
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_engine_gpu.py tests/test_registry.py tests/test_engine.py "tests/test_gpu_parity.py" -k "engine or registry or invoke or batched or diffusion_field or process or colony or division or lattice" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 6; }
tail -2 $O/pytest.log
timeout -k 10 600 python -u scripts/invoke_profile.py 500 2000 8000 32000 > $O/invoke_profile.log 2>&1 || { tail -20 $O/invoke_profile.log; exit 11; }
cat $O/invoke_profile.log
