# Round-4 final pass, part A: the whole GPU suite, smoke(), the drop-in rows.
set -o pipefail
timeout -k 10 1000 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/r04f_pytest.log 2>&1 || exit 1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r04f_smoke.log 2>&1 || exit 2
timeout -k 10 400 python bench.py --rows --reps 20 > gpurun_out/r04f_rows.json 2> gpurun_out/r04f_rows.err || exit 3
echo part A done
