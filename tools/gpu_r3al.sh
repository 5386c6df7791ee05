# halo wgrad conflict-free row layout (L=1): tests, per-layer A/B, same-box step A/B (L env)
set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_ops_gpu.py tests/test_swgrad_gpu.py tests/test_bf16_model_gpu.py -q -x -k "wgrad or bf16" --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r3al_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r3al_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/ab_wgrad_ma.py > gpurun_out/r3al_ab_wgrad.jsonl 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/r3al_ab_wgrad.jsonl
bash tools/ab_env_vals.sh RR_WGRAD_HALO_L 0 1 3 || exit 1
cat gpurun_out/ab_env_vals.txt
