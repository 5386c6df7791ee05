cd /root/repo
timeout -k 10 900 python -u -m pytest tests -m gpu -q --maxfail=8 --timeout 240 --timeout-method thread -rA > gpurun_out/${TAG:-r2a}_pytest.log 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python -u bench.py > gpurun_out/${TAG:-r2a}_bench.json 2> gpurun_out/${TAG:-r2a}_bench.err
rc2=$?
echo "bench rc=$rc2"
tail -c 3000 gpurun_out/${TAG:-r2a}_bench.json
exit $rc2
