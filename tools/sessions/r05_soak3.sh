# round-5 soak on the final tree (after the non-blocking source ring): new seeds for
# the random-descriptor tests, the two-rank random exchange and the random multi-rank programs
set -o pipefail
out=gpurun_out/r05soak3
mkdir -p $out
for s in 13 14 15 16 17 18; do
  GAAMD_FUZZ_SEED=$s timeout -k 10 300 python -u -m pytest tests/test_gpu_fuzz.py -m gpu -q --timeout 200 --timeout-method thread -p no:cacheprovider > $out/fuzz_$s.log 2>&1 || { tail -30 $out/fuzz_$s.log; exit 11; }
  echo "fuzz seed $s: $(tail -1 $out/fuzz_$s.log)"
done
for s in 51 52 53 54 55 56; do
  RDESC_SEED=$s RDESC_CASES=300 timeout -k 10 600 python -u -m pytest tests/test_multiproc.py -m gpu -q -k random_remote_descriptors --timeout 250 --timeout-method thread -p no:cacheprovider > $out/rdesc_$s.log 2>&1 || { tail -30 $out/rdesc_$s.log; exit 12; }
  echo "rdesc seed $s: $(tail -1 $out/rdesc_$s.log)"
done
for s in 61 62 63 64; do
  STRESS_SEED=$s timeout -k 10 600 python -u -m pytest tests/test_multiproc.py -m gpu -q -k "stress_random_programs and not one_pass" --timeout 250 --timeout-method thread -p no:cacheprovider > $out/stress_$s.log 2>&1 || { tail -30 $out/stress_$s.log; exit 13; }
  echo "stress seed $s: $(tail -1 $out/stress_$s.log)"
done
