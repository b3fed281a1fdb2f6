#!/bin/bash
# Host-side AddressSanitizer + UndefinedBehaviorSanitizer run of the CPU tests that drive the
# native host runtime (C++ reducer over gloo at world 2 and 8, forced world-1 reducer, bucket
# plans, bindings).  CPU only -- never on the GPU box (GPU sanitizers are not available there).
#   bash scripts/asan_cpu_tests.sh [pytest args...]
set -eo pipefail
R="$(cd "$(dirname "$0")/.." && pwd)"
cd "$R"
python build_native.py --sanitize > /tmp/pdt_asan_build.log 2>&1 || { tail -20 /tmp/pdt_asan_build.log; exit 1; }
SO=$(python -c "import build_native; print(build_native.asan_out_path())")
RT=$(ls /opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so | head -1)
# python itself is not instrumented: the runtime must be loaded first; CPython's arenas are
# reported as leaks at exit, so leak checking is off (use-after-free, overflows and UB stay on)
export LD_PRELOAD="$RT${LD_PRELOAD:+:$LD_PRELOAD}"
export ASAN_OPTIONS=detect_leaks=0:halt_on_error=1:abort_on_error=0
export UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1
export PDT_NATIVE_SO="$SO"
python -m pytest tests/test_ddp_cpu.py tests/test_plumbing_cpu.py -m "not gpu" -q -p no:cacheprovider "$@"
