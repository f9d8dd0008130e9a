#!/bin/bash
# Build the native loader with host sanitizers (ASan+UBSan, then TSan) and run the stress test.
# Host code only (GPU sanitizers are not available on this pool).  Usage: scripts/sanitize_native.sh <png dir> [iters]
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
DIR=${1:?png dir}
ITERS=${2:-30}
OUT=${TMPDIR:-/tmp}/tdl_sanitize
mkdir -p "$OUT"
SRC="$ROOT/tools/native/loader_stress.cpp $ROOT/csrc/runtime/loader.cpp"
g++ -std=c++17 -O1 -g -fno-omit-frame-pointer -fsanitize=address,undefined -fno-sanitize-recover=all \
    -I"$ROOT/csrc/runtime" $SRC -lz -pthread -o "$OUT/stress_asan"
ASAN_OPTIONS=detect_leaks=1 "$OUT/stress_asan" "$DIR" "$ITERS"
g++ -std=c++17 -O1 -g -fsanitize=thread -I"$ROOT/csrc/runtime" $SRC -lz -pthread -o "$OUT/stress_tsan"
TSAN_OPTIONS=halt_on_error=1 "$OUT/stress_tsan" "$DIR" "$ITERS"
