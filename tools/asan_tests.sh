#!/bin/bash
# Host sanitizer run (CPU only, this container): the library built with AddressSanitizer +
# UBSan (make asan) under the CPU tests of the parsers that read untrusted bytes: trace files
# (gzip + JSON and the binary cache), op-log files and mappings, the update wire format (RGA and
# Fugue: version-2 updates, the Fugue index rebuild, side columns).
set -e
cd "$(dirname "$0")/.."
make -s -C crdt-benches_amd asan
RT=$(/opt/rocm/lib/llvm/bin/clang -print-file-name=libclang_rt.asan-x86_64.so)
export CRDT_HIP_LIB=libcrdt_hip_asan.so
export ASAN_OPTIONS=detect_leaks=0:abort_on_error=1:halt_on_error=1
export UBSAN_OPTIONS=halt_on_error=1:print_stacktrace=1
LD_PRELOAD="$RT" python -m pytest tests/test_host.py tests/test_store.py tests/test_abi.py tests/test_fugue.py -q -m "not gpu" -p no:cacheprovider "$@"
