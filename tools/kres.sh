# per-kernel resource usage (VGPRs, SGPRs, SGPR spills, scratch, occupancy) of one source file
# usage: bash tools/kres.sh hygeia_amd/csrc/tg_kernels.hip
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-gpu-flush-denormals-to-zero \
  -fhip-fp32-correctly-rounded-divide-sqrt --offload-device-only -c -o /dev/null \
  -Rpass-analysis=kernel-resource-usage "$1" 2>&1 | awk -F': ' '
  /Function Name/ {n=$NF; sub(/ \[.*/, "", n); printf "\n%-70.70s", n}
  /VGPRs: / && !/AGPR/ {v=$NF; sub(/ \[.*/, "", v); printf " vgpr=%s", v}
  /TotalSGPRs/ {v=$NF; sub(/ \[.*/, "", v); printf " sgpr=%s", v}
  /SGPRs Spill/ {v=$NF; sub(/ \[.*/, "", v); printf " sspill=%s", v}
  /VGPRs Spill/ {v=$NF; sub(/ \[.*/, "", v); printf " vspill=%s", v}
  /ScratchSize/ {v=$NF; sub(/ \[.*/, "", v); printf " scratch=%s", v}
  /Occupancy/ {v=$NF; sub(/ \[.*/, "", v); printf " occ=%s", v}
  END {print ""}'
