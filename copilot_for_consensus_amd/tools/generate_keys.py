"""Write a JWT signing key pair into a secrets directory (reference auth/generate_keys.py).

    python -m copilot_for_consensus_amd.tools.generate_keys /run/secrets [--algorithm RS256|ES256]

Writes ``jwt_private_key`` (PKCS#8 PEM) and ``jwt_public_key`` (SubjectPublicKeyInfo PEM), the
secret names the local JWT signer's config reads (config/specs.py SECRET_FIELDS); existing files
are kept.  No `cryptography` dependency: security/jwt.py holds the RSA / P-256 and DER code.
"""
from __future__ import annotations

import argparse
import sys

from ..security.jwt import generate_keys


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("output_dir")
    ap.add_argument("--algorithm", default="RS256", choices=["RS256", "ES256"])
    ap.add_argument("--bits", type=int, default=2048)
    a = ap.parse_args(argv)
    priv, pub = generate_keys(a.output_dir, a.algorithm, a.bits)
    print(f"{priv}\n{pub}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
