# ladder at 512 bins (two pass-2 workgroups per CU): ladder tests, then C3 A/B
set -o pipefail
mkdir -p gpurun_out/r05p
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "ladder or c3" > gpurun_out/r05p/pytest.log 2>&1 || { tail -40 gpurun_out/r05p/pytest.log; exit 1; }
tail -2 gpurun_out/r05p/pytest.log
timeout -k 10 300 python -u tools/probe_ab.py 4 c3 > gpurun_out/r05p/ab_c3.log 2>&1 || { tail -20 gpurun_out/r05p/ab_c3.log; exit 1; }
tail -2 gpurun_out/r05p/ab_c3.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r05p/new -o run --output-format csv -- python tools/probe_prof.py auto 30 > gpurun_out/r05p/new.log 2>&1 || { tail -20 gpurun_out/r05p/new.log; exit 1; }
echo ok
