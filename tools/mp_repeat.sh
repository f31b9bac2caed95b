# repeat a multi-process worker mode; stop at the first failure (logs -> gpurun_out/fail)
MODE=${1:-ga}
N=${2:-4}
REPS=${3:-8}
for i in $(seq 1 $REPS); do
  timeout -k 10 60 bash tools/mp_debug.sh $MODE $N || { echo "run $i failed rc=$?"; mkdir -p gpurun_out/fail; cp gpurun_out/mp_${MODE}_*.log gpurun_out/fail/; exit 1; }
  echo "run $i ok"
done
