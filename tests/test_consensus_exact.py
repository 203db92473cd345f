"""CPU: the probabilistic batch modes stay out of consensus-relevant code.

`verify_bls_signature` (`/root/reference/utils/verify-bls-signatures/src/lib.rs:243-247`)
gives an exact, deterministic verdict per signature, and the audit pallet's
extrinsics depend on it.  The library's RLC modes accept an invalid batch with
a small probability (key-grouped: 2^-128 per check; distinct-key,
`CESS_BLS_F_RLC_DISTINCT`: 2^-63, `include/cess_bls.h`), so a node whose GPU
verdict came from one could disagree with wasm nodes.  This test asserts that
nothing on the node / runtime / pallet path -- the runtime host-function crate,
the batcher the patch adds, and every line the patch adds to the reference --
enables an RLC mode or calls an RLC entry point, and that the Rust crate's
default configuration is per-signature.
"""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
RUNTIME = os.path.join(ROOT, "utils", "cess-gpu-verify-runtime")
CRATE = os.path.join(ROOT, "utils", "verify-bls-signatures-gpu", "src", "lib.rs")

# anything that would select or call a probabilistic mode
RLC = re.compile(r"rlc|RLC|gt_product_is_one|MODE_RLC", re.I)


def _added_lines(patch):
    return [l[1:] for l in open(patch).read().splitlines() if l.startswith("+") and not l.startswith("+++")]


def _consensus_sources():
    out = {}
    for dirpath, _, files in os.walk(RUNTIME):
        for f in files:
            p = os.path.join(dirpath, f)
            if f.endswith(".rs"):
                out[os.path.relpath(p, ROOT)] = open(p).read().splitlines()
            elif f.endswith(".patch"):
                out[os.path.relpath(p, ROOT) + " (added lines)"] = _added_lines(p)
    return out


def test_consensus_path_never_selects_an_rlc_mode():
    srcs = _consensus_sources()
    assert any(k.endswith(".patch (added lines)") for k in srcs) and any("gpu_batcher.rs" in k for k in srcs)
    hits = [(k, i + 1, l.strip()) for k, lines in srcs.items() for i, l in enumerate(lines)
            if RLC.search(l) and not l.strip().startswith(("//", "///", "//!"))]
    assert not hits, hits


def test_crate_default_config_is_per_signature():
    src = open(CRATE).read()
    m = re.search(r"impl Default for Config \{.*?Config \{(.*?)\}", src, re.S)
    assert m, "Config::default not found"
    fields = dict(kv.split(":", 1) for kv in (x.strip() for x in m.group(1).replace("\n", " ").split(",")) if ":" in kv)
    assert fields["rlc"].strip() == "false" and fields["rlc_distinct"].strip() == "false", fields
    # the runtime state is built from the crate's Config (its callers pass
    # Config::default() or their own): no code path in the runtime crate sets a mode
    rt = open(os.path.join(RUNTIME, "src", "lib.rs")).read()
    assert "rlc" not in rt.lower()
