# Final check of the tree as committed: the whole GPU suite and smoke().
set -o pipefail
timeout -k 10 1000 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/r04final_pytest.log 2>&1 || exit 1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04final_smoke.log 2>&1 || exit 2
echo final ok
