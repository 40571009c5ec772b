#!/bin/bash
# Host-code sanitizers: build the native arrival collector + its self test with
# AddressSanitizer/UndefinedBehaviorSanitizer (g++, host only; GPU ASan is not available on the
# MI355X pool) and run it.  Usage: bash tools/sanitize_host.sh [outdir]
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=${1:-$ROOT/build/sanitize}
mkdir -p "$OUT"
ROCM=${ROCM_PATH:-/opt/rocm}
g++ -std=c++17 -O1 -g -fno-omit-frame-pointer -fsanitize=address,undefined -fno-sanitize-recover=undefined \
    -D__HIP_PLATFORM_AMD__=1 -I"$ROCM/include" -I"$ROOT/csrc/runtime" \
    "$ROOT/csrc/runtime/collector.cpp" "$ROOT/csrc/runtime/collector_selftest.cpp" \
    -L"$ROCM/lib" -Wl,-rpath,"$ROCM/lib" -lamdhip64 -o "$OUT/collector_selftest_asan"
ASAN_OPTIONS=detect_leaks=1:abort_on_error=1 UBSAN_OPTIONS=print_stacktrace=1 "$OUT/collector_selftest_asan"
