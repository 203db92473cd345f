//! Known-answer tests of the drop-in crate, on a box with cargo and an MI355X.
//! NOT COMPILED in this repository's image (no cargo/rustc); the same vectors
//! run through the C ABI in tests/test_oracle.py (oracle) and
//! tests/test_gpu_parity.py (GPU) on every round.
//!
//! Vectors: the reference crate's KATs (utils/verify-bls-signatures/tests/
//! tests.rs:19-112 -- two valid triples, the cross-swapped rejections, the
//! G1 non-subgroup and G2 off-curve rejections, the IC threshold signature, the
//! sign KAT), plus this crate's additions (batch, deserialize-only, random keys).
use ic_verify_bls_signature_gpu::*;

fn h(s: &str) -> Vec<u8> {
    (0..s.len()).step_by(2).map(|i| u8::from_str_radix(&s[i..i + 2], 16).unwrap()).collect()
}

struct Triple {
    sig: Vec<u8>,
    msg: Vec<u8>,
    key: Vec<u8>,
}

fn state_root_triples() -> [Triple; 2] {
    [
        Triple {
            sig: h("ace9fcdd9bc977e05d6328f889dc4e7c99114c737a494653cb27a1f55c06f4555e0f160980af5ead098acc195010b2f7"),
            msg: h("0d69632d73746174652d726f6f74e6c01e909b4923345ce5970962bcfe3004bfd8474a21dae28f50692502f46d90"),
            key: h(concat!("814c0e6ec71fab583b08bd81373c255c3c371b2e84863c98a4f1e08b74235d14fb5d9c0cd546d9685f913a0c0b2cc534",
                           "1583bf4b4392e467db96d65b9bb4cb717112f8472e0d5a4d14505ffd7484b01291091c5f87b98883463f98091a0baaae")),
        },
        Triple {
            sig: h("89a2be21b5fa8ac9fab1527e041327ce899d7da971436a1f2165393947b4d942365bfe5488710e61a619ba48388a21b1"),
            msg: h("0d69632d73746174652d726f6f74b294b418b11ebe5dd7dd1dcb099e4e0372b9a42aef7a7a37fb4f25667d705ea9"),
            key: h(concat!("9933e1f89e8a3c4d7fdcccdbd518089e2bd4d8180a261f18d9c247a52768ebce98dc7328a39814a8f911086a1dd50cbe",
                           "015e2a53b7bf78b55288893daa15c346640e8831d72a12bdedd979d28470c34823b8d1c3f4795d9c3984a247132e94fe")),
        },
    ]
}

#[test]
fn reference_triples_verify_and_cross_swaps_fail() {
    let [a, b] = state_root_triples();
    assert!(verify_bls_signature(&a.sig, &a.msg, &a.key).is_ok());
    assert!(verify_bls_signature(&b.sig, &b.msg, &b.key).is_ok());
    assert!(verify_bls_signature(&b.sig, &a.msg, &a.key).is_err());
    assert!(verify_bls_signature(&a.sig, &b.msg, &b.key).is_err());
}

#[test]
fn non_subgroup_signature_and_off_curve_key_fail() {
    let [a, _] = state_root_triples();
    let mut sig = a.sig.clone();
    *sig.last_mut().unwrap() = 0xf8;          // on the curve, not in G1
    assert!(verify_bls_signature(&sig, &a.msg, &a.key).is_err());
    assert_eq!(Signature::deserialize(&sig), Err(InvalidSignature::InvalidPoint));
    let mut key = a.key.clone();
    *key.last_mut().unwrap() = 0xad;          // x^3 + 4(1 + u) is not a square in Fp2
    assert!(verify_bls_signature(&a.sig, &a.msg, &key).is_err());
    assert_eq!(PublicKey::deserialize(&key), Err(InvalidPublicKey::InvalidPoint));
}

#[test]
fn ic_threshold_signature_verifies() {
    let key = h(concat!("87033f48fd8f327ff5d164e85af31433c6a8c73fc5a65bad5d472127205c73c5168a45e862f5af6d0da5676df45d0a5f",
                        "1293a530d5498f812a34a280f6bef869e4ca9b7c275554456d8770733d72ac4006777382fa541873fe002adb12184268"));
    let msg = h(concat!("e751fdb69185002b13c8d2954c7d0c39546402ecdde9c2a9a2c624293535a5ca2f560a582f705580448fbe1ccdc0e86af3",
                        "ba4c487a7f73bc9c312556"));
    let sig = h("98733cc2b312d5787cd4dba6ea0e19a1f1850b9e8c6d5112f12e12db8e7413a4ecb4096c23730566c67d9b2694e4e179");
    assert!(verify_bls_signature(&sig, &msg, &key).is_ok());
    assert!(PublicKey::deserialize(&key).unwrap().verify(&msg, &Signature::deserialize(&sig).unwrap()).is_ok());
}

#[test]
fn signing_kat_pins_hash_to_g1() {
    let sk = PrivateKey::deserialize(&h("6f3977f6051e184b2c412daa1b5c0115ef7ab347cac8d808ffa2c26bd0658243")).unwrap();
    let msg = h(concat!("50484522ad8aede64ec7f86b9273b7ed3940481acf93cdd40a2b77f2be2734a14012b2492b6363b12adaeaf055c573e4611b",
                        "085d2e0fe2153d72453a95eaebf350ac3ba6a26ba0bc79f4c0bf5664dfdf5865f69f7fc6b58ba7d068e8"));
    let want = h("8f7ad830632657f7b3eae17fd4c3d9ff5c13365eea8d33fd0a1a6d8fbebc5152e066bb0ad61ab64e8a8541c8e3f96de9");
    assert_eq!(sk.sign(&msg).serialize().to_vec(), want);
}

#[test]
fn random_keys_sign_verify_and_round_trip() {
    for i in 0..30u8 {
        let sk = PrivateKey::random();
        let pk = sk.public_key();
        let msg = [i; 24];
        let sig = sk.sign(&msg);
        assert!(pk.verify(&msg, &sig).is_ok());
        assert_eq!(PrivateKey::deserialize(&sk.serialize()).unwrap(), sk);
        assert_eq!(PublicKey::deserialize(&pk.serialize()).unwrap(), pk);
        assert_eq!(Signature::deserialize(&sig.serialize()).unwrap(), sig);
    }
}

#[test]
fn batch_codes_follow_reference_precedence() {
    let [a, b] = state_root_triples();
    let short = &a.sig[..47];
    let v = verify_batch(&[(&a.sig, &a.msg, &a.key), (&b.sig, &a.msg, &a.key), (short, &a.msg, &a.key),
                           (&a.sig, &a.msg, &a.key[..95])]);
    assert_eq!(v.codes, vec![0, 5, 1, 3]);
    assert!(v.ok(0) && !v.ok(1) && !v.ok(2) && !v.ok(3));
}

#[test]
fn verdict_cache_serves_repeats() {
    let [a, b] = state_root_triples();
    let cache = VerdictCache::new(1024).unwrap();
    let recs: [(&[u8], &[u8], &[u8]); 2] = [(&a.sig, &a.msg, &a.key), (&b.sig, &a.msg, &a.key)];
    let (codes, _, st) = cache.verify(None, &recs);
    assert_eq!(codes, vec![0xff, 0xff]);            // no verifier: unavailable, nothing cached
    assert!(st.is_err() && cache.len() == 0);
    let mut v = Verifier::new(&Config::default()).unwrap();
    let (codes, stats, st) = cache.verify(Some(&mut v), &recs);
    assert!(st.is_ok() && codes == vec![0, 5] && stats.verified == 2);
    let (codes, stats, _) = cache.verify(None, &recs);
    assert!(codes == vec![0, 5] && stats.hits == 2);
}
