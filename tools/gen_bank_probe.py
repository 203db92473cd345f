# Generates tools/bank_probe_body.inc: v_mad_u64_u32 streams with the operand
# VGPRs fixed in the asm text, so the register-file bank of every operand
# (VGPR index mod 4) is chosen: 8 independent accumulator pairs per stream.
# Usage: python3 tools/gen_bank_probe.py > tools/bank_probe_body.inc
CASES = {
    # name: (a, b, accumulator base registers; acc j = v[base+2j : base+2j+1])
    "nocf": (35, 34, 40),   # a bank 3, b bank 2, acc banks 0/1
    "a_acchi": (33, 34, 40),  # a bank 1 = acc hi bank
    "ab_same": (32, 36, 40),  # a, b and acc lo all bank 0
    "all_b0": (36, 44, 40),   # a, b bank 0; acc lo bank 0 (3-way)
}
out = []
for name, (a, b, base) in CASES.items():
    lines = []
    for q in range(64):
        j = q % 8
        lines.append(f"v_mad_u64_u32 v[{base + 2*j}:{base + 2*j + 1}], vcc, v{a}, v{b}, v[{base + 2*j}:{base + 2*j + 1}]")
    clob = sorted({f'"v{a}"', f'"v{b}"'} | {f'"v{base + k}"' for k in range(16)})
    s = "\\n\\t".join(lines)
    out.append(f'#define BANK_{name} asm volatile("{s}" ::: {", ".join(clob)}, "vcc");')
    out.append(f'#define BANK_INIT_{name} asm volatile("v_mov_b32 v{a}, %0\\n\\tv_mov_b32 v{b}, %1" :: "v"(aa), "v"(bb) : "v{a}", "v{b}");')
print("\n".join(out))
