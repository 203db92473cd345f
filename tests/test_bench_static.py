"""CPU: bench.py has no reference to an undefined name in any function (a
static check: symtable scopes against the module's own definitions and the
builtins), so a mode the default run does not exercise (rsa, sign, rlc,
keyed, adversarial) cannot die on a NameError on the GPU box."""
import builtins
import os
import symtable

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _undefined(path):
    src = open(path).read()
    top = symtable.symtable(src, path, "exec")
    module_names = {s.get_name() for s in top.get_symbols() if s.is_assigned() or s.is_imported()}
    module_names |= {c.get_name() for c in top.get_children()}
    bad = []

    def walk(t, chain):
        for s in t.get_symbols():
            if not s.is_referenced():
                continue
            n = s.get_name()
            if s.is_local() or s.is_parameter() or s.is_free() or s.is_imported():
                continue
            if s.is_global() or s.is_declared_global():
                if n not in module_names and not hasattr(builtins, n) and n not in ("__file__", "__name__"):
                    bad.append(f"{'.'.join(chain)}: {n}")
        for c in t.get_children():
            walk(c, chain + [c.get_name()])

    for c in top.get_children():
        walk(c, [c.get_name()])
    return bad


def test_bench_has_no_undefined_names():
    assert _undefined(os.path.join(ROOT, "bench.py")) == []


def test_graft_entry_has_no_undefined_names():
    assert _undefined(os.path.join(ROOT, "__graft_entry__.py")) == []
