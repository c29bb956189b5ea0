set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ "${SKIP_TESTS:-0}" != 1 ]; then
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_din.py tests/test_train.py -rf > gpurun_out/pt_dinfused.log 2>&1
rc=$?; tail -3 gpurun_out/pt_dinfused.log; [ $rc -eq 0 ] || exit $rc
fi
R=$(pwd); export PYTHONPATH=$R; cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_dintrain" -o run --output-format csv -- python3 "$R/scripts/prof_din_train.py" 6 > "$R/gpurun_out/prof_dintrain.log" 2>&1
rc=$?; grep -v "^W2026\|simple_timer" "$R/gpurun_out/prof_dintrain.log" | tail -8; exit $rc
