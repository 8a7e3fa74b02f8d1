#!/bin/bash
# Host-side sanitizer run (SURVEY.md §5 "race detection / sanitizers"): the C ABI (argument
# validation, host merge, blob layout), the C++ WordPiece / char tokenizers and the host
# logic, built with ASan + UBSan (host code only: `make asan`, no device code) and driven
# by the CPU test files that exercise them.  No GPU.
set -eo pipefail
cd "$(dirname "$0")/.."
make -C mediquery-rag_amd/csrc asan -j8 > /dev/null
RT=$(/opt/rocm/lib/llvm/bin/clang -print-file-name=libclang_rt.asan-x86_64.so)
export MQ_LIB_PATH=$PWD/mediquery-rag_amd/csrc/build_asan/libmqhip_asan.so
# leaks: the Python interpreter itself is not leak-clean; UBSan findings abort the run
export ASAN_OPTIONS=detect_leaks=0:halt_on_error=1:abort_on_error=1
export UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1
LD_PRELOAD=$RT python -m pytest -q -p no:cacheprovider "$@" \
  tests/test_tokenizer_native.py tests/test_abi.py tests/test_host_logic.py
