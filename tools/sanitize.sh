#!/bin/bash
# Build and run the host-runtime self-test under sanitizers (host code only;
# GPU sanitizers are not available on this pool).
#   tools/sanitize.sh [asan|tsan|all]   -> exit 0 iff every selected build passes
set -u
cd "$(dirname "$0")/.."
mode="${1:-all}"
out=build/sanitize
mkdir -p "$out"
srcs="csrc/runtime/selftest.cpp csrc/runtime/lz4.cpp csrc/runtime/zfp_rev.cpp csrc/runtime/zvc.cpp csrc/runtime/framing.cpp"
rc=0
if [ "$mode" = asan ] || [ "$mode" = all ]; then
  g++ -std=c++17 -O1 -g -fno-omit-frame-pointer -fsanitize=address,undefined -fno-sanitize-recover=undefined \
      -pthread -Icsrc/runtime $srcs -o "$out/selftest_asan" || exit 2
  ASAN_OPTIONS=detect_leaks=1:abort_on_error=1 UBSAN_OPTIONS=print_stacktrace=1 "$out/selftest_asan" || rc=1
fi
if [ "$mode" = tsan ] || [ "$mode" = all ]; then
  g++ -std=c++17 -O1 -g -fsanitize=thread -pthread -Icsrc/runtime $srcs -o "$out/selftest_tsan" || exit 2
  TSAN_OPTIONS=halt_on_error=1 "$out/selftest_tsan" || rc=1
fi
exit $rc
