#!/bin/bash
# The CPU test suite over AddressSanitizer + UBSan builds of the host code
# ("Race detection / sanitizers"): libxrt_host.so and
# xrt_main (make -C simpleraytracing_amd/csrc SAN=1 -> lib/san/) and the
# oracle (make -C oracle SAN=1 -> oracle/san/).  Python is not instrumented, so
# the sanitizer runtimes are preloaded; leak checking is off (the interpreter's
# own allocations).  Device code is never sanitised (no GPU ASan on this pool).
# Usage: tools/san_check.sh [pytest args and test paths]   (CPU only; default: every CPU test)
set -eo pipefail
cd "$(dirname "$0")/.."
make -C simpleraytracing_amd/csrc SAN=1 >/dev/null
make -C oracle SAN=1 >/dev/null
ASAN=$(gcc -print-file-name=libasan.so)
UBSAN=$(gcc -print-file-name=libubsan.so)
export LD_PRELOAD="$ASAN:$UBSAN"
export ASAN_OPTIONS=detect_leaks=0:verify_asan_link_order=0:abort_on_error=1
export UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1
export XRT_HOST_LIB=$PWD/simpleraytracing_amd/lib/san/libxrt_host.so
export XRT_ORACLE_LIB=$PWD/oracle/san/liboracle.so
export XRT_ORACLE_NO_REF=1
export XRT_MAIN=$PWD/simpleraytracing_amd/lib/san/xrt_main
ARGS=("$@")
case " $* " in *" tests/"*) ;; *) ARGS=(tests "${ARGS[@]}") ;; esac
python -m pytest -q -m "not gpu" -p no:cacheprovider --ignore=tests/test_sanitizers.py "${ARGS[@]}"
