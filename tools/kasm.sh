# device asm of one kernel instantiation: bash tools/kasm.sh <source> <mangled-name-prefix> <out.s>
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-gpu-flush-denormals-to-zero \
  -fhip-fp32-correctly-rounded-divide-sqrt --offload-device-only -S -o /tmp/kasm_all.s "$1" 2>/dev/null
s=$(grep -n "^$2" /tmp/kasm_all.s | head -1 | cut -d: -f1)
e=$(awk -v s=$s 'NR>s && /^\.Lfunc_end/ {print NR; exit}' /tmp/kasm_all.s)
awk -v s=$s -v e=$e 'NR>=s && NR<=e' /tmp/kasm_all.s > "$3"
wc -l "$3"
