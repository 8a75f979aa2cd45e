#!/bin/bash
# Build the native index builders with ASan + UBSan into a standalone driver
# and fuzz them (host-code sanitizers).  CPU only.
#   tools/sanitize/run_native.sh [iterations]
set -euo pipefail
ROOT="$(cd "$(dirname "$0")/../.." && pwd)"
OUT="$ROOT/build/sanitize"
mkdir -p "$OUT"
PYINC=$(python3 -c 'import sysconfig; print(sysconfig.get_paths()["include"])')
PBINC=$(python3 -c 'import pybind11; print(pybind11.get_include())')
PYLIB=$(python3 -c 'import sysconfig; print(sysconfig.get_config_var("LIBDIR"))')
PYVER=$(python3 -c 'import sysconfig; print(sysconfig.get_config_var("LDVERSION"))')
BIN="$OUT/native_asan"
if [ ! -x "$BIN" ] || [ "$ROOT/csrc/native/index_helpers.cpp" -nt "$BIN" ] || \
   [ "$ROOT/csrc/native/sanitize/driver.cpp" -nt "$BIN" ]; then
  ${CXX:-g++} -std=c++17 -O1 -g -fno-omit-frame-pointer -fsanitize=address,undefined \
      -fno-sanitize-recover=undefined -I"$PYINC" -I"$PBINC" \
      "$ROOT/csrc/native/index_helpers.cpp" "$ROOT/csrc/native/sanitize/driver.cpp" \
      -L"$PYLIB" -lpython"$PYVER" -o "$BIN"
fi
# leak checking is off: CPython and numpy keep interned objects until exit
ASAN_OPTIONS=detect_leaks=0:abort_on_error=0:halt_on_error=1 \
UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1 \
PYTHONHOME=$(python3 -c 'import sys; print(sys.base_prefix)') \
PYTHONPATH=$(python3 -c 'import numpy, os; print(os.path.dirname(os.path.dirname(numpy.__file__)))') \
    "$BIN" "$ROOT/tools/sanitize/fuzz_native.py" "${1:-40}"
