# Generates tools/issue_probe_body.inc: each probe group is ONE asm statement, so the
# hazard recognizer puts no s_nop between the instructions (it does after every
# separate inline asm).  Usage: python3 tools/gen_issue_probe.py > tools/issue_probe_body.inc
ops = {
 "mad": ("v_mad_u64_u32 %{j}, vcc, %[a], %[b], %{j}", "y"),
 "and": ("v_and_b32 %{j}, %{j}, %[a]", "x"),
 "lshr64": ("v_lshrrev_b64 %{j}, 1, %{j}", "y"),
 "madand": ("v_mad_u64_u32 %{j}, vcc, %[a], %[b], %{j}\\n\\tv_and_b32 %{k}, %{k}, %[a]", "yx"),
}
out = []
for name, (tmpl, kind) in ops.items():
    for ch in (1, 2, 4, 8, 16):
        if name == "madand" and ch > 8: continue
        lines = []
        per = 32 if name != "madand" else 16
        for q in range(per):
            j = q % ch
            if kind == "yx":
                lines.append(tmpl.format(j=j, k=ch + j))
            else:
                lines.append(tmpl.format(j=j))
        s = "\\n\\t".join(lines)
        if kind == "y": opnds = ", ".join(f'"+v"(y[{j}])' for j in range(ch))
        elif kind == "x": opnds = ", ".join(f'"+v"(x[{j}])' for j in range(ch))
        else: opnds = ", ".join([f'"+v"(y[{j}])' for j in range(ch)] + [f'"+v"(x[{j}])' for j in range(ch)])
        out.append(f'  if (OP == {list(ops).index(name)} && CH == {ch}) asm volatile("{s}" : {opnds} : [a] "v"(a), [b] "v"(b) : "vcc");')
print("\n".join(out))
