# round 3 session 21: completion seen through a tail flag kernel (one lane stores a tag to
# pinned host memory; the host spins on it) against hipStreamSynchronize, for one launch (a
# blocking comex_accs) and 20 (the value region's close); bare HIP, the H shape, interleaved;
# plus the torch-runtime IPC hang repro (does it still hang?)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/s21
export TMPDIR=/tmp
timeout -k 10 200 ./tools/completion_probe 20 300 3 > gpurun_out/s21/tail_flag.jsonl 2> gpurun_out/s21/tail.err || exit 1
cat gpurun_out/s21/tail_flag.jsonl
timeout -k 10 200 ./tools/completion_probe 20 300 3 > gpurun_out/s21/tail_flag_2.jsonl 2> gpurun_out/s21/tail2.err || exit 1
cat gpurun_out/s21/tail_flag_2.jsonl
REPRO_TORCH=1 REPRO_KEEP=1 timeout -k 10 90 python -u tools/malloc_repro.py 1 2 > gpurun_out/s21/malloc_repro_torch.log 2>&1
echo "torch-first repro rc=$?"; tail -5 gpurun_out/s21/malloc_repro_torch.log
