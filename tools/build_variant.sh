# An A/B build of the same sources with extra flags into hygeia_amd/lib/var_<tag>/
# (select it with HYG_LIB_PATH=hygeia_amd/lib/var_<tag>/libhygeia_amd.so).
# usage: bash tools/build_variant.sh <tag> -DNAME=VALUE ...
tag=$1; shift
D=hygeia_amd/lib/var_$tag
mkdir -p $D
F="--offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=off -fno-gpu-flush-denormals-to-zero -fhip-fp32-correctly-rounded-divide-sqrt -w"
for s in capi.cpp tg_kernels.hip sg_kernels.hip dmp_kernels.hip bed_kernels.hip pre_kernels.hip; do
  /opt/rocm/bin/hipcc $F "$@" -c hygeia_amd/csrc/$s -o $D/$s.o &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $D/libhygeia_amd.so $D/*.o && rm -f $D/*.o && echo $D/libhygeia_amd.so
# the sources it was built from (tools/gpu_final.sh refuses a stale variant)
python3 -c "from hygeia_amd import build; print(build.source_hash())" > $D/source_hash
