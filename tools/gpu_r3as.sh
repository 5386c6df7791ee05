# round-end rehearsal: smoke(), cfg5 inference and cfg2 SimpleUNet on the final build
set -o pipefail
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3as_smoke.log 2>&1 || exit 1
tail -2 gpurun_out/r3as_smoke.log
timeout -k 10 300 python tools/bench_inference.py --images 4096 > gpurun_out/r3as_inf_bf16.json 2> gpurun_out/r3as_inf.err || exit 1
cat gpurun_out/r3as_inf_bf16.json
timeout -k 10 300 python tools/bench_cfg2.py > gpurun_out/r3as_cfg2.jsonl 2> gpurun_out/r3as_cfg2.err || exit 1
cat gpurun_out/r3as_cfg2.jsonl
