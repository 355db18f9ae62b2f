#!/bin/bash
# Host-side sanitizer builds of the native runtime (no GPU code): the PS service + TensorBundle
# writer under ThreadSanitizer and AddressSanitizer/UBSan, driven by csrc/tests/ps_stress.cc.
#   tools/build_sanitizers.sh [thread|address|all]   -> build/san/ps_stress_{tsan,asan}
set -euo pipefail
cd "$(dirname "$0")/.."
mkdir -p build/san
SRCS="csrc/tests/ps_stress.cc csrc/ps/server.cc"
# LLVM's runtime: gcc-11's libtsan lacks the pthread_cond_clockwait interceptor that
# std::condition_variable::wait_for uses, and reports false "double lock" errors.
CXX=${CXX:-/opt/rocm/lib/llvm/bin/clang++}
COMMON="-std=c++17 -g -O1 -fno-omit-frame-pointer -Icsrc/include -pthread"
which=${1:-all}
if [ "$which" = thread ] || [ "$which" = all ]; then
  $CXX $COMMON -fsanitize=thread $SRCS -o build/san/ps_stress_tsan
fi
if [ "$which" = address ] || [ "$which" = all ]; then
  $CXX $COMMON -fsanitize=address,undefined $SRCS -o build/san/ps_stress_asan
fi
echo "built build/san/ps_stress_*"
