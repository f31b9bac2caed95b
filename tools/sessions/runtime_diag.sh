set -o pipefail
mkdir -p gpurun_out/r05d1
export COMEX_AMD_DEBUG=2 COMEX_AMD_ALLOW_HIP_MISMATCH=1 REPRO_DUMP_S=30
for alloc in ipc vmm; do
  echo "=== torch first, allocator $alloc" 
  REPRO_TORCH=1 REPRO_KEEP=1 COMEX_AMD_SEGMENT_ALLOC=$alloc timeout -k 10 45 python3 -u tools/malloc_repro.py 1 2 > gpurun_out/r05d1/torch_$alloc.log 2>&1
  echo "rc=$?" >> gpurun_out/r05d1/torch_$alloc.log
  tail -4 gpurun_out/r05d1/torch_$alloc.log
  rc=$(tail -1 gpurun_out/r05d1/torch_$alloc.log)
done
echo "=== library first, vmm"
REPRO_KEEP=1 COMEX_AMD_SEGMENT_ALLOC=vmm timeout -k 10 45 python3 -u tools/malloc_repro.py 1 2 > gpurun_out/r05d1/lib_vmm.log 2>&1; echo "rc=$?" >> gpurun_out/r05d1/lib_vmm.log
tail -3 gpurun_out/r05d1/lib_vmm.log
