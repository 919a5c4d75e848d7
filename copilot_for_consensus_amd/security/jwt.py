"""JWT signing/verification without third-party crypto (PyJWT / cryptography are not in the image).

Reference: adapters/copilot_jwt_signer (LocalJWTSigner RSA/EC/HMAC, local_signer.py:214-271) and
copilot_auth/jwt_manager.py (mint :154, validate :265, JWKS :322).

* HS256 -- stdlib ``hmac``.
* ES256 -- ECDSA over NIST P-256 with SHA-256, deterministic nonces (RFC 6979), Jacobian point
  arithmetic on Python integers, JWK ``kty=EC, crv=P-256, x, y``; signatures in the JOSE raw
  ``r || s`` form (RFC 7518 §3.4).
* RS256 -- RSASSA-PKCS1-v1_5 with SHA-256 implemented on Python integers: key generation
  (Miller-Rabin primes, e = 65537), CRT signing, public verification, JWK / JWKS export
  (``kty=RSA, n, e, kid``) so services can verify tokens from the auth service's JWKS exactly as
  with the reference.  (Timing side channels are out of scope for this signer; use the
  key-vault signer in hostile environments.)
"""
from __future__ import annotations

import base64
import hashlib
import hmac
import json
import secrets as _secrets
import time
import uuid
from abc import ABC, abstractmethod
from typing import Any


class JWTError(ValueError):
    pass


def b64u(b: bytes) -> str:
    return base64.urlsafe_b64encode(b).rstrip(b"=").decode()


def b64u_dec(s: str) -> bytes:
    return base64.urlsafe_b64decode(s + "=" * (-len(s) % 4))


def _int_to_b(n: int, length: int | None = None) -> bytes:
    length = length or max(1, (n.bit_length() + 7) // 8)
    return n.to_bytes(length, "big")


# ------------------------------------------------------------------------------------ RSA math

_SMALL_PRIMES = [p for p in range(3, 2000, 2) if all(p % q for q in range(3, int(p ** 0.5) + 1, 2))]


def _is_probable_prime(n: int, rounds: int = 40) -> bool:
    if n < 2:
        return False
    for p in _SMALL_PRIMES:
        if n % p == 0:
            return n == p
    d, r = n - 1, 0
    while d % 2 == 0:
        d //= 2
        r += 1
    for _ in range(rounds):
        a = _secrets.randbelow(n - 3) + 2
        x = pow(a, d, n)
        if x in (1, n - 1):
            continue
        for _ in range(r - 1):
            x = pow(x, 2, n)
            if x == n - 1:
                break
        else:
            return False
    return True


def _gen_prime(bits: int) -> int:
    while True:
        c = _secrets.randbits(bits) | (1 << (bits - 1)) | (1 << (bits - 2)) | 1
        if _is_probable_prime(c):
            return c


class RSAKey:
    def __init__(self, n: int, e: int, d: int | None = None, p: int | None = None, q: int | None = None):
        self.n, self.e, self.d, self.p, self.q = n, e, d, p, q
        self.size = (n.bit_length() + 7) // 8
        if p and q and d:
            self.dp, self.dq, self.qinv = d % (p - 1), d % (q - 1), pow(q, -1, p)

    @classmethod
    def generate(cls, bits: int = 2048, e: int = 65537) -> "RSAKey":
        while True:
            p, q = _gen_prime(bits // 2), _gen_prime(bits // 2)
            if p == q:
                continue
            phi = (p - 1) * (q - 1)
            try:
                d = pow(e, -1, phi)
            except ValueError:
                continue
            return cls(p * q, e, d, p, q)

    _SHA256_PREFIX = bytes.fromhex("3031300d060960864801650304020105000420")

    def _emsa(self, msg: bytes) -> int:
        t = self._SHA256_PREFIX + hashlib.sha256(msg).digest()
        em = b"\x00\x01" + b"\xff" * (self.size - len(t) - 3) + b"\x00" + t
        return int.from_bytes(em, "big")

    def sign(self, msg: bytes) -> bytes:
        if self.d is None:
            raise JWTError("private key required")
        m = self._emsa(msg)
        if self.p:
            s1, s2 = pow(m, self.dp, self.p), pow(m, self.dq, self.q)
            s = s2 + self.q * ((self.qinv * (s1 - s2)) % self.p)
            # a fault in either half-exponentiation leaks a factor of n through gcd(s^e - m, n)
            # (Boneh-DeMillo-Lipton): check the signature before it leaves
            if pow(s, self.e, self.n) != m:
                raise JWTError("RSA-CRT signature failed its self-check")
        else:
            s = pow(m, self.d, self.n)
        return _int_to_b(s, self.size)

    def verify(self, msg: bytes, sig: bytes) -> bool:
        if len(sig) != self.size:
            return False
        return pow(int.from_bytes(sig, "big"), self.e, self.n) == self._emsa(msg)

    def public_jwk(self, kid: str) -> dict:
        return {"kty": "RSA", "use": "sig", "alg": "RS256", "kid": kid, "n": b64u(_int_to_b(self.n)),
                "e": b64u(_int_to_b(self.e))}

    @classmethod
    def from_jwk(cls, jwk: dict) -> "RSAKey":
        return cls(int.from_bytes(b64u_dec(jwk["n"]), "big"), int.from_bytes(b64u_dec(jwk["e"]), "big"))

    def private_json(self) -> str:
        return json.dumps({k: hex(getattr(self, k)) for k in ("n", "e", "d", "p", "q")})

    @classmethod
    def from_private_json(cls, s: str) -> "RSAKey":
        d = {k: int(v, 16) for k, v in json.loads(s).items()}
        return cls(d["n"], d["e"], d["d"], d.get("p"), d.get("q"))


# ------------------------------------------------------------------------------------ P-256 math

_P = 0xffffffff00000001000000000000000000000000ffffffffffffffffffffffff
_A = _P - 3
_B = 0x5ac635d8aa3a93e7b3ebbd55769886bc651d06b0cc53b0f63bce3c3e27d2604b
_N = 0xffffffff00000000ffffffffffffffffbce6faada7179e84f3b9cac2fc632551
_G = (0x6b17d1f2e12c4247f8bce6e563a440f277037d812deb33a0f4a13945d898c296,
      0x4fe342e2fe1a7f9b8ee7eb4a7c0f9e162bce33576b315ececbb6406837bf51f5)


def _jdouble(P):
    X, Y, Z = P
    if Y == 0:
        return (0, 1, 0)
    YY = Y * Y % _P
    S = 4 * X * YY % _P
    ZZ = Z * Z % _P
    M = 3 * (X - ZZ) * (X + ZZ) % _P          # a = -3
    X3 = (M * M - 2 * S) % _P
    return (X3, (M * (S - X3) - 8 * YY * YY) % _P, 2 * Y * Z % _P)


def _jadd(P, Q):
    if P[2] == 0:
        return Q
    if Q[2] == 0:
        return P
    X1, Y1, Z1 = P
    X2, Y2, Z2 = Q
    Z1Z1, Z2Z2 = Z1 * Z1 % _P, Z2 * Z2 % _P
    U1, U2 = X1 * Z2Z2 % _P, X2 * Z1Z1 % _P
    S1, S2 = Y1 * Z2 * Z2Z2 % _P, Y2 * Z1 * Z1Z1 % _P
    if U1 == U2:
        return _jdouble(P) if S1 == S2 else (0, 1, 0)
    H, R = (U2 - U1) % _P, (S2 - S1) % _P
    HH = H * H % _P
    HHH = H * HH % _P
    V = U1 * HH % _P
    X3 = (R * R - HHH - 2 * V) % _P
    return (X3, (R * (V - X3) - S1 * HHH) % _P, H * Z1 * Z2 % _P)


def _jmul(k: int, pt) -> tuple[int, int] | None:
    """k * pt by a Montgomery ladder over a fixed 258-bit schedule: k is first replaced by k + N
    or k + 2N (same point, since N * pt = O), so the top bit and the number of steps never depend
    on the scalar, and every step does one add and one double whatever the bit is (the bit only
    selects which register receives which result)."""
    k %= _N
    k += _N
    if k.bit_length() <= 256:
        k += _N
    R0, R1 = (0, 1, 0), (pt[0], pt[1], 1)
    for i in range(257, -1, -1):
        b = (k >> i) & 1
        S, D = _jadd(R0, R1), _jdouble(R1 if b else R0)
        R0, R1 = (S, D) if b else (D, S)
    R = R0
    if R[2] == 0:
        return None
    zi = pow(R[2], -1, _P)
    return (R[0] * zi * zi % _P, R[1] * zi * zi * zi % _P)


def _on_curve(x: int, y: int) -> bool:
    return 0 <= x < _P and 0 <= y < _P and (y * y - (x * x * x + _A * x + _B)) % _P == 0


def _rfc6979_k(d: int, h1: bytes) -> int:
    """Deterministic nonce (RFC 6979 §3.2) for P-256 / SHA-256."""
    x = _int_to_b(d, 32)
    h = _int_to_b(int.from_bytes(h1, "big") % _N, 32)
    V, K = b"\x01" * 32, b"\x00" * 32
    K = hmac.new(K, V + b"\x00" + x + h, hashlib.sha256).digest()
    V = hmac.new(K, V, hashlib.sha256).digest()
    K = hmac.new(K, V + b"\x01" + x + h, hashlib.sha256).digest()
    V = hmac.new(K, V, hashlib.sha256).digest()
    while True:
        V = hmac.new(K, V, hashlib.sha256).digest()
        k = int.from_bytes(V, "big")
        if 1 <= k < _N:
            return k
        K = hmac.new(K, V + b"\x00", hashlib.sha256).digest()
        V = hmac.new(K, V, hashlib.sha256).digest()


class ECKey:
    """P-256 key: private scalar ``d`` (optional) and public point ``(x, y)``."""

    def __init__(self, x: int, y: int, d: int | None = None):
        if not _on_curve(x, y):
            raise JWTError("point not on P-256")
        self.x, self.y, self.d = x, y, d

    @classmethod
    def generate(cls) -> "ECKey":
        d = _secrets.randbelow(_N - 1) + 1
        x, y = _jmul(d, _G)
        return cls(x, y, d)

    def sign(self, msg: bytes) -> bytes:
        if self.d is None:
            raise JWTError("private key required")
        h = hashlib.sha256(msg).digest()
        e = int.from_bytes(h, "big")
        while True:
            k = _rfc6979_k(self.d, h)
            r = _jmul(k, _G)[0] % _N
            s = pow(k, -1, _N) * (e + r * self.d) % _N
            if r and s:
                return _int_to_b(r, 32) + _int_to_b(s, 32)
            h = hashlib.sha256(h).digest()   # practically unreachable; keep determinism

    def verify(self, msg: bytes, sig: bytes) -> bool:
        if len(sig) != 64:
            return False
        r, s = int.from_bytes(sig[:32], "big"), int.from_bytes(sig[32:], "big")
        if not (1 <= r < _N and 1 <= s < _N):
            return False
        e = int.from_bytes(hashlib.sha256(msg).digest(), "big")
        w = pow(s, -1, _N)
        u1, u2 = e * w % _N, r * w % _N
        P1, P2 = _jmul(u1, _G), _jmul(u2, (self.x, self.y))
        if P1 is None or P2 is None:
            pt = P1 or P2
        else:
            R = _jadd((P1[0], P1[1], 1), (P2[0], P2[1], 1))
            if R[2] == 0:
                return False
            zi = pow(R[2], -1, _P)
            pt = (R[0] * zi * zi % _P, 0)
        return pt is not None and pt[0] % _N == r

    def public_jwk(self, kid: str) -> dict:
        return {"kty": "EC", "crv": "P-256", "use": "sig", "alg": "ES256", "kid": kid,
                "x": b64u(_int_to_b(self.x, 32)), "y": b64u(_int_to_b(self.y, 32))}

    def public_pem(self) -> str:
        spki = bytes.fromhex("3059301306072a8648ce3d020106082a8648ce3d030107034200") + b"\x04" + \
            _int_to_b(self.x, 32) + _int_to_b(self.y, 32)
        body = base64.encodebytes(spki).decode().replace("\n", "")
        lines = [body[i:i + 64] for i in range(0, len(body), 64)]
        return "-----BEGIN PUBLIC KEY-----\n" + "\n".join(lines) + "\n-----END PUBLIC KEY-----\n"

    @classmethod
    def from_jwk(cls, jwk: dict) -> "ECKey":
        if jwk.get("crv") != "P-256":
            raise JWTError("only P-256 EC keys are supported")
        d = int.from_bytes(b64u_dec(jwk["d"]), "big") if "d" in jwk else None
        return cls(int.from_bytes(b64u_dec(jwk["x"]), "big"), int.from_bytes(b64u_dec(jwk["y"]), "big"), d)

    def private_json(self) -> str:
        return json.dumps({"kty": "EC", "crv": "P-256", "x": b64u(_int_to_b(self.x, 32)),
                           "y": b64u(_int_to_b(self.y, 32)), "d": b64u(_int_to_b(self.d, 32))})


# ------------------------------------------------------------------------------------ PEM / DER
# Just enough ASN.1 DER for the key files the reference's auth/generate_keys.py writes (PKCS#8
# PrivateKeyInfo + SubjectPublicKeyInfo, via `cryptography`) and for OpenSSL's PKCS#1 / SEC1
# forms, so a deployment's existing /run/secrets/jwt_private_key works unchanged.

_OID_RSA = bytes.fromhex("2a864886f70d010101")          # 1.2.840.113549.1.1.1 rsaEncryption
_OID_EC = bytes.fromhex("2a8648ce3d0201")                # 1.2.840.10045.2.1 id-ecPublicKey
_OID_P256 = bytes.fromhex("2a8648ce3d030107")            # 1.2.840.10045.3.1.7 prime256v1


def _der_read(buf: bytes, pos: int = 0) -> tuple[int, bytes, int]:
    """One TLV at ``pos``: (tag, value, position after it)."""
    if pos + 2 > len(buf):
        raise JWTError("truncated DER")
    tag, ln = buf[pos], buf[pos + 1]
    pos += 2
    if ln & 0x80:
        n = ln & 0x7F
        if n == 0 or n > 4 or pos + n > len(buf):
            raise JWTError("bad DER length")
        ln = int.from_bytes(buf[pos:pos + n], "big")
        pos += n
    if pos + ln > len(buf):
        raise JWTError("truncated DER")
    return tag, buf[pos:pos + ln], pos + ln


def _der_items(seq: bytes) -> list[tuple[int, bytes]]:
    out, pos = [], 0
    while pos < len(seq):
        tag, val, pos = _der_read(seq, pos)
        out.append((tag, val))
    return out


def _der(tag: int, val: bytes) -> bytes:
    n = len(val)
    if n < 0x80:
        return bytes([tag, n]) + val
    lb = _int_to_b(n)
    return bytes([tag, 0x80 | len(lb)]) + lb + val


def _der_int(v: int) -> bytes:
    b = _int_to_b(v) if v else b"\x00"
    return _der(0x02, (b"\x00" + b) if b[0] & 0x80 else b)


def _pem_decode(text: str) -> tuple[str, bytes]:
    lines = [ln.strip() for ln in text.strip().splitlines() if ln.strip()]
    if len(lines) < 2 or not lines[0].startswith("-----BEGIN ") or not lines[-1].startswith("-----END "):
        raise JWTError("not a PEM block")
    return lines[0][11:].rstrip("-").strip(), base64.b64decode("".join(lines[1:-1]))


def _pem_encode(label: str, der: bytes) -> str:
    body = base64.b64encode(der).decode()
    return f"-----BEGIN {label}-----\n" + "\n".join(body[i:i + 64] for i in range(0, len(body), 64)) + \
        f"\n-----END {label}-----\n"


def _ints(seq: bytes) -> list[int]:
    return [int.from_bytes(v, "big") for t, v in _der_items(seq) if t == 0x02]


def load_pem_key(text: str) -> "RSAKey | ECKey":
    """A PEM private or public key: PKCS#8 / PKCS#1 / SEC1 private keys, SPKI / PKCS#1 public keys
    (RSA, or EC on P-256)."""
    label, der = _pem_decode(text)
    tag, body, _ = _der_read(der)
    if tag != 0x30:
        raise JWTError("PEM body is not a DER SEQUENCE")
    items = _der_items(body)
    if label == "RSA PRIVATE KEY":
        v = _ints(body)
        return RSAKey(v[1], v[2], v[3], v[4], v[5])
    if label == "RSA PUBLIC KEY":
        n, e = _ints(body)[:2]
        return RSAKey(n, e)
    if label == "EC PRIVATE KEY":
        return _ec_from_sec1(body)
    if label == "PRIVATE KEY":          # PKCS#8 PrivateKeyInfo {version, algorithm, privateKey}
        alg = _der_items(items[1][1])
        inner = _der_read(items[2][1])[1]
        if alg[0][1] == _OID_RSA:
            v = _ints(inner)
            return RSAKey(v[1], v[2], v[3], v[4], v[5])
        if alg[0][1] == _OID_EC and len(alg) > 1 and alg[1][1] == _OID_P256:
            return _ec_from_sec1(inner)
        raise JWTError("unsupported PKCS#8 key algorithm (RSA and EC P-256 only)")
    if label == "PUBLIC KEY":           # SubjectPublicKeyInfo {algorithm, BIT STRING}
        alg = _der_items(items[0][1])
        bits = items[1][1][1:]          # skip the unused-bits byte
        if alg[0][1] == _OID_RSA:
            n, e = _ints(_der_read(bits)[1])[:2]
            return RSAKey(n, e)
        if alg[0][1] == _OID_EC and bits[:1] == b"\x04" and len(bits) == 65:
            return ECKey(int.from_bytes(bits[1:33], "big"), int.from_bytes(bits[33:], "big"))
        raise JWTError("unsupported public key algorithm (RSA and EC P-256 only)")
    raise JWTError(f"unsupported PEM block {label!r}")


def _ec_from_sec1(seq: bytes) -> "ECKey":
    """ECPrivateKey {version, privateKey OCTET STRING, [0] params, [1] publicKey}."""
    items = _der_items(seq)
    d = int.from_bytes(items[1][1], "big")
    x, y = _jmul(d, _G)
    return ECKey(x, y, d)


def rsa_private_pem(k: "RSAKey") -> str:
    """PKCS#8 PEM (the format of the reference's generate_keys.py)."""
    dp, dq, qi = k.d % (k.p - 1), k.d % (k.q - 1), pow(k.q, -1, k.p)
    rsa = _der(0x30, b"".join(_der_int(v) for v in (0, k.n, k.e, k.d, k.p, k.q, dp, dq, qi)))
    alg = _der(0x30, _der(0x06, _OID_RSA) + _der(0x05, b""))
    return _pem_encode("PRIVATE KEY", _der(0x30, _der_int(0) + alg + _der(0x04, rsa)))


def rsa_public_pem(k: "RSAKey") -> str:
    alg = _der(0x30, _der(0x06, _OID_RSA) + _der(0x05, b""))
    pub = _der(0x30, _der_int(k.n) + _der_int(k.e))
    return _pem_encode("PUBLIC KEY", _der(0x30, alg + _der(0x03, b"\x00" + pub)))


def ec_private_pem(k: "ECKey") -> str:
    sec1 = _der(0x30, _der_int(1) + _der(0x04, _int_to_b(k.d, 32)) +
                _der(0xA1, _der(0x03, b"\x00\x04" + _int_to_b(k.x, 32) + _int_to_b(k.y, 32))))
    alg = _der(0x30, _der(0x06, _OID_EC) + _der(0x06, _OID_P256))
    return _pem_encode("PRIVATE KEY", _der(0x30, _der_int(0) + alg + _der(0x04, sec1)))


def _load_private(text: str, kind: type):
    """A private key given as PEM (any form load_pem_key reads) or as this module's JSON."""
    if text.lstrip().startswith("-----BEGIN"):
        key = load_pem_key(text)
    else:
        key = RSAKey.from_private_json(text) if kind is RSAKey else ECKey.from_jwk(json.loads(text))
    if not isinstance(key, kind) or key.d is None:
        raise JWTError(f"expected a {kind.__name__[:2]} private key")
    return key


def _check_public(key, public_key: str | None) -> None:
    """The configured public key must be the private key's own (a mismatched pair would mint
    tokens that no verifier holding the published key accepts)."""
    if not public_key:
        return
    text = public_key.strip()
    if text.startswith("-----BEGIN"):
        pub = load_pem_key(text)
    else:
        try:
            jwk = json.loads(text)
        except ValueError:
            raise JWTError("public_key is neither PEM nor a JSON / JWK key") from None
        if isinstance(jwk, dict) and "keys" in jwk and jwk["keys"]:   # a JWKS: its first key
            jwk = jwk["keys"][0]
        if not isinstance(jwk, dict):
            raise JWTError("public_key JSON is not a JWK object")
        kty = jwk.get("kty") or ("RSA" if "n" in jwk else "EC" if "x" in jwk else None)
        if kty == "RSA":
            pub = RSAKey.from_jwk(jwk)
        elif kty == "EC":
            pub = ECKey.from_jwk(jwk)
        else:
            raise JWTError(f"public_key JWK has an unsupported kty {kty!r}")
    if type(pub) is not type(key):
        raise JWTError("public_key does not match private_key (different key types)")
    same = (pub.n, pub.e) == (key.n, key.e) if isinstance(key, RSAKey) else (pub.x, pub.y) == (key.x, key.y)
    if not same:
        raise JWTError("public_key does not match private_key")


def generate_keys(output_dir, algorithm: str = "RS256", bits: int = 2048) -> tuple:
    """Write ``jwt_private_key`` / ``jwt_public_key`` (PEM) into a secrets directory -- the local
    secret provider's layout (reference auth/generate_keys.py writes the same PKCS#8 / SPKI PEM).
    Existing files are kept.  Returns the two paths."""
    from pathlib import Path
    out = Path(output_dir)
    out.mkdir(parents=True, exist_ok=True)
    priv, pub = out / "jwt_private_key", out / "jwt_public_key"
    if not (priv.exists() and pub.exists()):
        if algorithm.upper().startswith("ES"):
            k = ECKey.generate()
            priv.write_text(ec_private_pem(k))
            pub.write_text(k.public_pem())
        else:
            k = RSAKey.generate(bits)
            priv.write_text(rsa_private_pem(k))
            pub.write_text(rsa_public_pem(k))
        priv.chmod(0o600)
    return priv, pub


# ------------------------------------------------------------------------------------ signers

class JWTSigner(ABC):
    algorithm: str
    key_id: str

    @abstractmethod
    def sign(self, message: bytes) -> bytes: ...

    @abstractmethod
    def verify(self, message: bytes, signature: bytes) -> bool: ...

    def get_public_key_jwk(self) -> dict | None:
        return None

    def health_check(self) -> bool:
        return True


class HMACSigner(JWTSigner):
    algorithm = "HS256"

    def __init__(self, secret_key: str | bytes | None = None, key_id: str = "default", **_):
        if not secret_key:
            secret_key = _secrets.token_hex(32)
        self.key = secret_key.encode() if isinstance(secret_key, str) else secret_key
        self.key_id = key_id

    def sign(self, message):
        return hmac.new(self.key, message, hashlib.sha256).digest()

    def verify(self, message, signature):
        return hmac.compare_digest(self.sign(message), signature)


class RSASigner(JWTSigner):
    algorithm = "RS256"

    def __init__(self, private_key: str | RSAKey | None = None, key_id: str = "default", bits: int = 2048,
                 public_key: str | None = None, **_):
        if isinstance(private_key, RSAKey):
            self.key = private_key
        elif private_key:
            self.key = _load_private(private_key, RSAKey)
        else:
            self.key = RSAKey.generate(bits)   # tests / explicit ephemeral use; config requires a key
        _check_public(self.key, public_key)
        self.key_id = key_id

    def sign(self, message):
        return self.key.sign(message)

    def verify(self, message, signature):
        return self.key.verify(message, signature)

    def get_public_key_jwk(self):
        return self.key.public_jwk(self.key_id)


class ECSigner(JWTSigner):
    algorithm = "ES256"

    def __init__(self, private_key: str | ECKey | None = None, key_id: str = "default", public_key: str | None = None,
                 **_):
        if isinstance(private_key, ECKey):
            self.key = private_key
        elif private_key:
            self.key = _load_private(private_key, ECKey)
        else:
            self.key = ECKey.generate()
        _check_public(self.key, public_key)
        self.key_id = key_id

    def sign(self, message):
        return self.key.sign(message)

    def verify(self, message, signature):
        return self.key.verify(message, signature)

    def get_public_key_jwk(self):
        return self.key.public_jwk(self.key_id)


def create_jwt_signer(cfg=None, **overrides) -> JWTSigner:
    kw = {k: v for k, v in dict(getattr(cfg, "driver_config", {}) or {}).items() if v is not None}
    kw.update(overrides)
    alg = str(kw.pop("algorithm", "HS256")).upper()
    if alg == "HS256":
        return HMACSigner(**kw)
    if alg == "RS256":
        return RSASigner(**kw)
    if alg == "ES256":
        return ECSigner(**kw)
    raise JWTError(f"unsupported JWT algorithm {alg}")


# ------------------------------------------------------------------------------------ tokens

def encode(claims: dict, signer: JWTSigner) -> str:
    header = {"alg": signer.algorithm, "typ": "JWT", "kid": signer.key_id}
    signing_input = f"{b64u(json.dumps(header, separators=(',', ':')).encode())}." \
                    f"{b64u(json.dumps(claims, separators=(',', ':')).encode())}"
    return f"{signing_input}.{b64u(signer.sign(signing_input.encode()))}"


def decode_unverified(token: str) -> tuple[dict, dict]:
    try:
        h, p, _ = token.split(".")
        return json.loads(b64u_dec(h)), json.loads(b64u_dec(p))
    except Exception as e:
        raise JWTError("malformed token") from e


def decode(token: str, verify_key, audience: str | list[str] | None = None, issuer: str | None = None,
           leeway: int = 90, now: float | None = None) -> dict:
    """Verify signature (a signer, an RSAKey, or a JWKS dict) and registered claims."""
    header, claims = decode_unverified(token)
    h, p, s = token.split(".")
    msg = f"{h}.{p}".encode()
    sig = b64u_dec(s)
    alg = header.get("alg")
    if isinstance(verify_key, dict) and "keys" in verify_key:
        jwk = next((k for k in verify_key["keys"] if k.get("kid") == header.get("kid")), None)
        if jwk is None:
            raise JWTError("unknown kid")
        verify_key = ECKey.from_jwk(jwk) if jwk.get("kty") == "EC" else RSAKey.from_jwk(jwk)
    if isinstance(verify_key, RSAKey):
        ok = alg == "RS256" and verify_key.verify(msg, sig)
    elif isinstance(verify_key, ECKey):
        ok = alg == "ES256" and verify_key.verify(msg, sig)
    elif isinstance(verify_key, JWTSigner):
        ok = alg == verify_key.algorithm and verify_key.verify(msg, sig)
    else:
        raise JWTError("no verification key")
    if not ok:
        raise JWTError("invalid signature")
    now = time.time() if now is None else now
    if "exp" in claims and now > claims["exp"] + leeway:
        raise JWTError("token expired")
    if "nbf" in claims and now < claims["nbf"] - leeway:
        raise JWTError("token not yet valid")
    if audience is not None:
        aud = claims.get("aud")
        auds = aud if isinstance(aud, list) else [aud]
        want = audience if isinstance(audience, list) else [audience]
        if not set(auds) & set(want):
            raise JWTError("audience mismatch")
    if issuer is not None and claims.get("iss") != issuer:
        raise JWTError("issuer mismatch")
    return claims


class JWTManager:
    """Mints service tokens and publishes the JWKS (copilot_auth/jwt_manager.py:35)."""

    def __init__(self, signer: JWTSigner, issuer: str = "copilot-auth", audience: str = "copilot-for-consensus",
                 default_expiry: int = 1800):
        self.signer, self.issuer, self.audience, self.default_expiry = signer, issuer, audience, default_expiry

    def mint_token(self, subject: str, claims: dict | None = None, expires_in: int | None = None,
                   audience: str | None = None) -> str:
        now = int(time.time())
        c: dict[str, Any] = {"iss": self.issuer, "sub": subject, "aud": audience or self.audience, "iat": now,
                             "nbf": now, "exp": now + int(expires_in or self.default_expiry), "jti": str(uuid.uuid4())}
        c.update(claims or {})
        return encode(c, self.signer)

    def validate_token(self, token: str, audience: str | None = None, max_skew: int = 90) -> dict:
        return decode(token, self.signer, audience=audience or self.audience, issuer=self.issuer, leeway=max_skew)

    def get_jwks(self) -> dict:
        jwk = self.signer.get_public_key_jwk()
        return {"keys": [jwk] if jwk else []}
