# per region between consecutive s_memtime markers of a kernel's asm: counts of
# VALU / SALU / LDS ops, lgkmcnt waits, vmcnt waits, exec-mask branches, barriers
# usage: bash tools/asm_regions.sh /tmp/asm/f.s
awk '
/s_memtime/ { if (n++) printf "region %2d line %6d: valu %5d salu %5d ds %4d lgkm-waits %4d vm-waits %3d execz-br %4d barriers %2d readlane %4d\n", n-1, start, v, s, d, lw, vw, br, b, rl; start=NR; v=s=d=lw=vw=br=b=rl=0; next }
/^[ \t]*v_readlane|^[ \t]*v_writelane/ {rl++}
/^[ \t]*v_/ {v++} /^[ \t]*s_/ {s++} /^[ \t]*ds_/ {d++}
/s_waitcnt.*lgkmcnt/ {lw++} /s_waitcnt.*vmcnt/ {vw++} /s_cbranch_execz|s_cbranch_execnz/ {br++} /s_barrier/ {b++}
' "$1"
