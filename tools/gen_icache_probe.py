# generates tools/icache_probe_body.inc: straight-line mad+and streams of
# several lengths (one asm statement per 64 instructions)
out = []
for name, n in (("L64", 64), ("L4K", 4096), ("L32K", 32768), ("L64K", 65536)):
    blocks = []
    for b in range(n // 64):
        lines = []
        for q in range(32):
            j = q % 8
            lines.append(f"v_mad_u64_u32 %{j}, vcc, %[a], %[b], %{j}")
            lines.append(f"v_and_b32 %{8 + j}, %{8 + j}, %[a]")
        s = "\\n\\t".join(lines)
        opnds = ", ".join([f'"+v"(y[{j}])' for j in range(8)] + [f'"+v"(x[{j}])' for j in range(8)])
        blocks.append(f'    asm volatile("{s}" : {opnds} : [a] "v"(a), [b] "v"(b) : "vcc");')
    out.append(f"#define BODY_{name} \\\n" + " \\\n".join(b for b in blocks))
print("\n".join(out))
