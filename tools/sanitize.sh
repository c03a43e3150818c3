# Host-code sanitizer pass (sanitizers row): the CPU suite
# (pytest -m "not gpu") with AddressSanitizer + UndefinedBehaviorSanitizer, no
# recovery (the first report fails the run), over
#   - the CPU oracle (oracle/*.c and the shared include/hyg_arith.h,
#     hyg_model.h, hyg_sg_model.h, hyg_sg_pe.h it compiles): make SAN=1;
#   - the product library's host code (capi.cpp's argument checks, slot locks,
#     workspace layouts, the host-side model tables from the same shared
#     headers, the BED formatter): every translation unit built with
#     -Xarch_host -fsanitize=... (device code is not instrumented; GPU
#     sanitizers are not available on the pool).
# Both builds use the ROCm clang so one ASan runtime serves the process; it is
# preloaded into python (which is not instrumented itself; leak detection off,
# the interpreter keeps its arenas). CPU only: no GPU is touched.
# usage: bash tools/sanitize.sh [pytest args]   (default: tests -m "not gpu")
set -eu
cd "$(dirname "$0")/.."
LLVM=/opt/rocm/lib/llvm
RT=$(ls $LLVM/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so | head -1)
make -C oracle SAN=1 CC=$LLVM/bin/clang -s
D=hygeia_amd/lib/var_san
mkdir -p $D
F="--offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=off -fno-gpu-flush-denormals-to-zero
   -fhip-fp32-correctly-rounded-divide-sqrt -w
   -Xarch_host -O1 -Xarch_host -g -Xarch_host -fno-omit-frame-pointer
   -Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined -Xarch_host -fno-sanitize-recover=all"
pids=""
for s in capi.cpp tg_kernels.hip sg_kernels.hip dmp_kernels.hip bed_kernels.hip pre_kernels.hip; do
  /opt/rocm/bin/hipcc $F -c hygeia_amd/csrc/$s -o $D/$s.o &
  pids="$pids $!"
done
for p in $pids; do wait $p; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined \
  -shared-libsan -o $D/libhygeia_amd.so $D/*.o
rm -f $D/*.o
echo "sanitizer builds: oracle/build_san/, $D/libhygeia_amd.so (runtime $RT)"
# the builds really are instrumented (ASan reports and UBSan handlers referenced)
for f in $D/libhygeia_amd.so oracle/build_san/libtg_oracle.so oracle/build_san/libsg_oracle.so; do
  n=$(nm -D $f | grep -c "__asan_report\|__ubsan_handle" || true)
  [ "$n" -gt 0 ] || { echo "$f is not instrumented"; exit 1; }
done
if [ $# -eq 0 ]; then set -- tests -m "not gpu"; fi
export HYG_ORACLE_DIR=build_san HYG_LIB_PATH=$PWD/$D/libhygeia_amd.so
export ASAN_OPTIONS=detect_leaks=0:abort_on_error=1:halt_on_error=1:allocator_may_return_null=1
export UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1
LD_PRELOAD=$RT python -m pytest -x -q -p no:cacheprovider "$@"
