"""cess_amd — MI355X-native batch verifier for the BLS12-381 signature path of
CESS (utils/verify-bls-signatures).  See DESIGN.md."""
from .bls import (  # noqa: F401
    CODE_NAMES, Context, DeserializeError, DeviceUnavailable, InvalidPrivateKey, InvalidPublicKey,
    InvalidSignature, PrivateKey, PublicKey, Result, Signature, Verdicts, default_context, load_library,
    verify_batch, verify_bls_signature,
)
