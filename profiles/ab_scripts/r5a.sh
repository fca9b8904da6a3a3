set -uo pipefail
O=gpurun_out/r5a; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_multiprocess.py -m gpu -k "weak_graph or as_shard" > $O/tests.txt 2>&1; rc=$?
tail -5 $O/tests.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || exit 1
python -c "import json;d=json.load(open('$O/bench.json'));print(d['value'],d['stages_ms']);print(json.dumps(d['roofline'])[:1500]);print(d['step_floor']);print(json.dumps(d.get('gemm_legs')));print(d['cpu_baseline'])"
