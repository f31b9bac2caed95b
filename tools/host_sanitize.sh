#!/bin/bash
# Host-side AddressSanitizer + UBSan run of the CPU test suite (no GPU; GPU
# sanitizers are not available on the pool).  The g++ host objects of
# libga_amd.so (comex, armci, sched, bootstrap, wire), libga_amd_ga.so (ga) and
# libga_amd_diag.so are rebuilt with
# -fsanitize=address,undefined in a scratch tree, swapped in for the duration
# of the run, and the in-tree library is restored afterwards.  The hipcc
# objects stay uninstrumented (one ASan runtime per process: gcc's).
#
#   bash tools/host_sanitize.sh            # reports to /tmp/gaamd_asan/*.log
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
W=/tmp/gaamd_asan
rm -rf "$W" && mkdir -p "$W/pkg"
cp -r "$ROOT/include" "$W/" && cp -r "$ROOT/ga_amd/csrc" "$W/pkg/"
rm -f "$W"/pkg/csrc/*.o
mkdir -p "$W/lib"
make -s -C "$W/pkg/csrc" -j8 OUT="$W/lib/libga_amd.so" GA_OUT="$W/lib/libga_amd_ga.so" DIAG_OUT="$W/lib/libga_amd_diag.so" \
  CXXFLAGS="-O1 -g -fPIC -std=c++17 -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include -fsanitize=address,undefined -fno-omit-frame-pointer"
mkdir -p "$W/real"
for l in libga_amd libga_amd_ga libga_amd_diag; do cp "$ROOT/ga_amd/$l.so" "$W/real/"; done
trap 'cp "$W"/real/*.so "$ROOT/ga_amd/"' EXIT
cp "$W"/lib/*.so "$ROOT/ga_amd/"
GCCLIB=$(dirname "$(gcc -print-file-name=libasan.so)")
cd "$ROOT"
# the tests that link a plain C program against the library (test_c_client_compiles_and_links,
# test_global_src_armci_calls_link, test_init_over_a_sub_communicator) cannot link an
# instrumented build without the sanitizer runtimes
LD_PRELOAD="$GCCLIB/libasan.so $GCCLIB/libubsan.so${LD_PRELOAD:+ $LD_PRELOAD}" \
ASAN_OPTIONS=detect_leaks=0:verify_asan_link_order=0:log_path=$W/asan \
UBSAN_OPTIONS=print_stacktrace=1:log_path=$W/ubsan \
  python -m pytest tests -q -m "not gpu" -p no:cacheprovider \
    --deselect tests/test_abi.py::test_c_client_compiles_and_links \
    --deselect "tests/test_abi.py::test_global_src_armci_calls_link[False]" \
    --deselect "tests/test_abi.py::test_global_src_armci_calls_link[True]" \
    --deselect tests/test_abi.py::test_init_over_a_sub_communicator \
    --deselect tests/test_abi.py::test_program_defining_ga_names_links
if ls "$W"/asan* "$W"/ubsan* >/dev/null 2>&1; then
  echo "sanitizer reports:"; ls "$W"/asan* "$W"/ubsan* 2>/dev/null; exit 1
fi
echo "host sanitizers: clean"
