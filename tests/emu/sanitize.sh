#!/bin/bash
# TEST-ONLY: build the engine's host emulation + the oracle as one executable under
# AddressSanitizer + UndefinedBehaviorSanitizer (host code only; no GPU) and run it.
# usage: tests/emu/sanitize.sh [outdir]     (exit status != 0 on any report or mismatch)
set -e
HERE=$(cd "$(dirname "$0")" && pwd)
OUT=${1:-/tmp/mt_sanitize}
mkdir -p "$OUT"
g++ -O1 -g -std=c++17 -pthread -Wno-unknown-pragmas -DMT_G_MWMIN=64 -DMT_BPC_CHECK=1 \
    -fsanitize=address,undefined -fno-sanitize-recover=all -fno-omit-frame-pointer \
    -o "$OUT/sanitize_driver" "$HERE/sanitize_driver.cpp" "$HERE/../../oracle/mtoracle.cpp"
ASAN_OPTIONS=verify_asan_link_order=0:halt_on_error=1:detect_stack_use_after_return=1 \
UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1 "$OUT/sanitize_driver"
