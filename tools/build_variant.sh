# builds hygeia_amd/lib/libhygeia_amd_<name>.so: the library with extra compiler flags on tg_kernels.hip
# usage: bash tools/build_variant.sh <name> <extra flags...>   (load it with HYG_LIB_PATH)
name=$1; shift
O=hygeia_amd/lib/obj
F="--offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=off -fno-gpu-flush-denormals-to-zero -fhip-fp32-correctly-rounded-divide-sqrt"
/opt/rocm/bin/hipcc $F "$@" -c hygeia_amd/csrc/tg_kernels.hip -o /tmp/tg_$name.o &&
objs=$(ls $O/*.o | grep -v tg_kernels) &&
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o hygeia_amd/lib/libhygeia_amd_$name.so /tmp/tg_$name.o $objs && echo built hygeia_amd/lib/libhygeia_amd_$name.so
