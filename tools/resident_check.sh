#!/bin/bash
# GPU: the service-mode tests (incl. the resident kernel), then the bench's service leg
OUT=gpurun_out/$1; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_service.py -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" $OUT/pytest.log | head -20; exit $rc; }
timeout -k 10 300 python -u bench.py --steps 1 --warmup 0 --no-steal --no-c3 --no-c5 --no-variants --no-latency > $OUT/bench.log 2>&1
rc=$?; grep '^{' $OUT/bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps(d['service']))"; exit $rc
