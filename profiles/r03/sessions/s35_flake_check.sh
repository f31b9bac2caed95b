# round 3 session 35: flakiness check of the final tree -- the whole GPU suite twice more in a
# row, then the random-program stress with 6 more seeds (one-pass everywhere and default)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/s35
mkdir -p $O
export TMPDIR=/tmp
for i in 1 2; do
  timeout -k 10 600 python -u -m pytest tests/ -v --timeout 480 --timeout-method thread -m gpu > $O/gpu_suite_$i.log 2>&1
  rc=$?; grep -E "FAILED|ERROR" $O/gpu_suite_$i.log | head; tail -1 $O/gpu_suite_$i.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
done
for seed in 21 22 23; do
  STRESS_SEED=$seed STRESS_OPS=1000 timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests/test_multiproc.py -k "test_stress_random_programs" > $O/stress_$seed.log 2>&1
  rc=$?; echo "seed $seed: $(tail -1 $O/stress_$seed.log)"; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
done
