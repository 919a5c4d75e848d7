"""JWT signing/verification (HS256 against the RFC 7515 A.1 vector, RS256, ES256), claim checks,
JWKS, secrets providers, role store, the OIDC login state machine and the bearer-token middleware.
Mirrors adapters/copilot_jwt_signer/tests, copilot_auth/tests (test_jwt_manager.py,
test_middleware.py, test_mock_provider.py), copilot_secrets/tests and auth/tests of the reference."""
from __future__ import annotations

import base64
import time

import pytest

from copilot_for_consensus_amd.security import jwt as J
from copilot_for_consensus_amd.security.auth import (AuthService, JWTMiddleware, MockIdentityProvider, RoleStore,
                                                     pkce_pair)
from copilot_for_consensus_amd.security.secrets import (EnvSecretProvider, LocalFileSecretProvider, SecretNotFoundError,
                                                        create_secret_provider)
from copilot_for_consensus_amd.storage.document_store import InMemoryDocumentStore


def _b64d(s):
    return base64.urlsafe_b64decode(s + "=" * (-len(s) % 4))


def test_hs256_rfc7515_appendix_a1_vector():
    key = _b64d("AyM1SysPpbyDfgZld3umj1qzKObwVMkoqQ-EstJQLr_T-1qS0gZH75aKtMN3Yj0iPS4hcgUuTwjAzZr1Z9CAow")
    signing_input = (b"eyJ0eXAiOiJKV1QiLA0KICJhbGciOiJIUzI1NiJ9."
                     b"eyJpc3MiOiJqb2UiLA0KICJleHAiOjEzMDA4MTkzODAsDQogImh0dHA6Ly9leGFtcGxlLmNvbS9pc19yb290Ijp0cnVlfQ")
    signer = J.HMACSigner(key)
    assert J.b64u(signer.sign(signing_input)) == "dBjftJeZ4CVP-mB92K27uhbUJU1p1r_wW1gFWFOEjXk"
    token = signing_input.decode() + ".dBjftJeZ4CVP-mB92K27uhbUJU1p1r_wW1gFWFOEjXk"
    claims = J.decode(token, signer, now=1300819380 - 10)
    assert claims["iss"] == "joe" and claims["http://example.com/is_root"] is True
    with pytest.raises(J.JWTError, match="expired"):
        J.decode(token, signer, now=1300819380 + 1000)


@pytest.mark.parametrize("alg", ["HS256", "RS256", "ES256"])
def test_sign_verify_roundtrip_and_tamper(alg):
    kw = {"bits": 1024} if alg == "RS256" else {}
    signer = J.create_jwt_signer(None, algorithm=alg, key_id="k1", **kw)
    mgr = J.JWTManager(signer, issuer="iss", audience="aud", default_expiry=60)
    tok = mgr.mint_token("user-1", {"roles": ["reader"]})
    claims = mgr.validate_token(tok)
    assert claims["sub"] == "user-1" and claims["roles"] == ["reader"] and claims["exp"] - claims["iat"] == 60
    h, p, s = tok.split(".")
    forged = J.b64u(b'{"sub":"admin","iss":"iss","aud":"aud","roles":["admin"]}')
    with pytest.raises(J.JWTError, match="signature"):
        J.decode(f"{h}.{forged}.{s}", signer)
    with pytest.raises(J.JWTError, match="audience"):
        mgr.validate_token(tok, audience="other")
    with pytest.raises(J.JWTError, match="issuer"):
        J.decode(tok, signer, issuer="someone-else")
    if alg != "HS256":
        jwks = mgr.get_jwks()
        assert jwks["keys"][0]["kid"] == "k1"
        assert J.decode(tok, jwks)["sub"] == "user-1"      # verify with only the public JWKS
        with pytest.raises(J.JWTError, match="kid"):
            J.decode(tok, {"keys": []})
    else:
        assert mgr.get_jwks() == {"keys": []}  # symmetric keys are never published


def test_algorithm_confusion_is_rejected():
    rs = J.RSASigner(bits=1024)
    tok = J.encode({"sub": "x"}, rs)
    # a token claiming HS256 must not verify against an RSA key (alg confusion)
    h, p, s = tok.split(".")
    hs_header = J.b64u(b'{"alg":"HS256","typ":"JWT","kid":"default"}')
    with pytest.raises(J.JWTError):
        J.decode(f"{hs_header}.{p}.{s}", rs.key)
    with pytest.raises(J.JWTError):
        J.decode("not.a.token", rs)
    with pytest.raises(J.JWTError):
        J.create_jwt_signer(None, algorithm="none")


def test_nbf_and_leeway():
    s = J.HMACSigner("k")
    now = time.time()
    tok = J.encode({"sub": "x", "nbf": now + 100, "exp": now + 200}, s)
    with pytest.raises(J.JWTError, match="not yet"):
        J.decode(tok, s, leeway=10)
    assert J.decode(tok, s, leeway=120)["sub"] == "x"


def test_rsa_key_serialisation_roundtrip():
    k = J.RSAKey.generate(1024)
    k2 = J.RSAKey.from_private_json(k.private_json())
    sig = k2.sign(b"msg")
    assert k.verify(b"msg", sig) and not k.verify(b"msg2", sig)
    pub = J.RSAKey.from_jwk(k.public_jwk("x"))
    assert pub.verify(b"msg", sig)


def test_ec_key_serialisation_and_pem():
    k = J.ECKey.generate()
    signer = J.ECSigner(k.private_json(), key_id="e")
    sig = signer.sign(b"m")
    assert len(sig) == 64 and k.verify(b"m", sig) and not k.verify(b"n", sig)
    assert k.public_pem().startswith("-----BEGIN PUBLIC KEY-----")


# ------------------------------------------------------------------ secrets
def test_local_file_secrets(tmp_path):
    (tmp_path / "jwt_private_key").write_text("s3cret\n")
    p = create_secret_provider("local", base_path=str(tmp_path))
    assert isinstance(p, LocalFileSecretProvider)
    assert p.get_secret("jwt_private_key") == "s3cret" and p.get_secret_bytes("jwt_private_key") == b"s3cret\n"
    assert p.secret_exists("jwt_private_key") and not p.secret_exists("nope")
    with pytest.raises(SecretNotFoundError):
        p.get_secret("nope")
    for bad in ("../etc/passwd", "a/b", "..", ""):
        with pytest.raises(ValueError):
            p.get_secret(bad)
        assert not p.secret_exists(bad)


def test_env_secrets():
    p = EnvSecretProvider(prefix="app-", env={"APP_DB_PASSWORD": "pw"})
    assert p.get_secret("db.password") == "pw" and p.secret_exists("db-password")
    with pytest.raises(SecretNotFoundError):
        p.get_secret("other")
    with pytest.raises(ValueError):
        create_secret_provider("vault9000")


# ------------------------------------------------------------------ roles + login flow
def _auth(first_admin=True):
    store = InMemoryDocumentStore()
    roles = RoleStore(store, first_user_auto_promotion=first_admin)
    mgr = J.JWTManager(J.HMACSigner("k"), issuer="copilot-auth", audience="copilot-for-consensus")
    return AuthService(mgr, roles, {"mock": MockIdentityProvider()}), roles, mgr


def test_role_store_lifecycle():
    _, roles, _ = _auth()
    admin = roles.ensure_user({"sub": "u1", "email": "a@x", "name": "Ann"})
    assert admin["roles"] == ["admin", "reader"] and admin["status"] == "approved"
    second = roles.ensure_user({"sub": "u2", "email": "b@x", "name": "Bob"})
    assert second["status"] == "pending" and [u["_id"] for u in roles.pending()[0]] == ["u2"]
    assert roles.assign("u2", ["reader", "contributor"])["roles"] == ["contributor", "reader"]
    assert roles.revoke("u2", ["contributor"])["roles"] == ["reader"]
    assert [u["_id"] for u in roles.search("BOB", "name")] == ["u2"]
    with pytest.raises(ValueError):
        roles.deny("u2")                              # approved: only pending requests can be denied
    roles.ensure_user({"sub": "u3", "name": "Cy"})
    roles.deny("u3")
    assert roles.roles("u3") == [] and roles.get("u3")["status"] == "denied"
    with pytest.raises(KeyError):
        roles.revoke("ghost", ["reader"])
    assert roles.assign("ghost", ["reader"])["status"] == "approved"   # assigning creates the record
    assert roles.ensure_user({"sub": "u1"})["roles"] == ["admin", "reader"]  # idempotent


def test_pkce_pair_is_s256():
    import hashlib
    v, c = pkce_pair()
    assert 43 <= len(v) <= 128 and c == J.b64u(hashlib.sha256(v.encode()).digest())


def test_login_flow_and_refresh():
    svc, roles, mgr = _auth()
    start = svc.initiate_login("mock")
    assert "state=" in start["authorization_url"]
    res = svc.handle_callback("mock-user", start["state"])
    claims = svc.validate_token(res["access_token"])
    assert claims["sub"] == "mock:mock-user" and claims["roles"] == ["admin", "reader"]
    with pytest.raises(PermissionError):
        svc.handle_callback("mock-user", start["state"])  # state is single-use
    with pytest.raises(PermissionError):
        svc.handle_callback("x", "forged-state")
    with pytest.raises(KeyError):
        svc.initiate_login("myspace")
    roles.revoke("mock:mock-user", ["admin"])
    roles.assign("mock:mock-user", ["reader"])
    refreshed = svc.validate_token(svc.refresh(res["access_token"])["access_token"])
    assert refreshed["roles"] == ["reader"]  # refresh picks up role changes


def test_state_expiry():
    svc, _, _ = _auth()
    svc.state_ttl = 0
    st = svc.initiate_login("mock")["state"]
    time.sleep(0.01)
    with pytest.raises(PermissionError):
        svc.handle_callback("c", st)


def test_middleware_roles_and_http_codes():
    from fastapi import Depends, FastAPI
    from fastapi.testclient import TestClient

    mgr = J.JWTManager(J.HMACSigner("k"), audience="copilot-for-consensus")
    mw = JWTMiddleware(verify_key=mgr.signer, required_roles=["admin"])
    app = FastAPI()

    @app.get("/secret")
    def secret(claims=Depends(mw.dependency())):
        return {"sub": claims["sub"]}

    c = TestClient(app)
    assert c.get("/secret").status_code == 401
    assert c.get("/secret", headers={"Authorization": "Bearer garbage"}).status_code == 401
    reader = mgr.mint_token("r", {"roles": ["reader"]})
    assert c.get("/secret", headers={"Authorization": f"Bearer {reader}"}).status_code == 403
    admin = mgr.mint_token("a", {"roles": ["admin"]})
    r = c.get("/secret", headers={"Authorization": f"Bearer {admin}"})
    assert r.status_code == 200 and r.json() == {"sub": "a"}
    other_aud = mgr.mint_token("a", {"roles": ["admin"]}, audience="elsewhere")
    assert c.get("/secret", headers={"Authorization": f"Bearer {other_aud}"}).status_code == 401


class _FakeOIDC:
    """OIDCProvider with the two HTTP calls stubbed out."""

    @staticmethod
    def make(token_resp: dict, userinfo: dict, scope: str = "openid email profile"):
        from copilot_for_consensus_amd.security.auth import OIDCProvider

        p = OIDCProvider("acme", "client-1", "secret", "https://app/cb", "https://idp/authorize", "https://idp/token",
                         "https://idp/userinfo", scope=scope)
        p._post = lambda url, data: dict(token_resp)
        p._get = lambda url, token: dict(userinfo)
        return p


def _id_token(claims: dict) -> str:
    import json

    def enc(d):
        return base64.urlsafe_b64encode(json.dumps(d).encode()).rstrip(b"=").decode()
    return f"{enc({'alg': 'RS256'})}.{enc(claims)}.sig"


def test_oidc_exchange_checks_nonce_audience_and_subject():
    ok = {"access_token": "at", "id_token": _id_token({"nonce": "n1", "aud": "client-1", "sub": "u"})}
    p = _FakeOIDC.make(ok, {"sub": "u", "email": "u@x"})
    assert p.exchange_code("c", "v", "n1")["sub"] == "acme:u"
    with pytest.raises(PermissionError, match="nonce"):
        p.exchange_code("c", "v", "other-nonce")
    bad_aud = {"access_token": "at", "id_token": _id_token({"nonce": "n1", "aud": ["someone-else"]})}
    with pytest.raises(PermissionError, match="audience"):
        _FakeOIDC.make(bad_aud, {"sub": "u"}).exchange_code("c", "v", "n1")
    # an OpenID provider that returns no id_token cannot prove the nonce
    with pytest.raises(PermissionError, match="id_token"):
        _FakeOIDC.make({"access_token": "at"}, {"sub": "u"}).exchange_code("c", "v", "n1")
    # plain OAuth (GitHub-style, no openid scope): no id_token expected
    gh = _FakeOIDC.make({"access_token": "at"}, {"id": 42, "login": "octo"}, scope="read:user")
    assert gh.exchange_code("c", "v", "n1") == {"sub": "acme:42", "email": None, "name": "octo", "provider": "acme"}
    # userinfo without sub / id must not collapse every such user into "acme:None"
    with pytest.raises(PermissionError, match="subject"):
        _FakeOIDC.make({"access_token": "at"}, {"email": "x@y"}, scope="read:user").exchange_code("c", "v", "n")


def test_oidc_discovery_and_jwks_verified_id_token():
    """Discovery fills the endpoints; the id_token is verified against the provider JWKS: signature,
    iss, aud, exp and nonce; an unknown kid triggers one JWKS refresh (key rotation)."""
    import time as _t

    from copilot_for_consensus_amd.security.auth import OIDCProvider
    k_old, k_new = J.RSAKey.generate(1024), J.RSAKey.generate(1024)
    jwks = {"keys": [k_old.public_jwk("old")]}
    fetched = []

    def fetch(url):
        fetched.append(url)
        if url.endswith("/.well-known/openid-configuration"):
            return {"issuer": "https://idp.example", "authorization_endpoint": "https://idp.example/auth",
                    "token_endpoint": "https://idp.example/token", "userinfo_endpoint": "https://idp.example/me",
                    "jwks_uri": "https://idp.example/jwks"}
        return {"keys": list(jwks["keys"])}

    def signed(key, kid, **claims):
        base = {"iss": "https://idp.example", "aud": "client-1", "sub": "u", "nonce": "n1",
                "exp": int(_t.time()) + 300}
        base.update(claims)
        return J.encode(base, J.RSASigner(key, key_id=kid))

    token = {"access_token": "at"}
    p = OIDCProvider("acme", "client-1", "secret", "https://app/cb", issuer="https://idp.example")
    p._fetch_json = fetch
    p._post = lambda url, data: dict(token)
    p._get = lambda url, tok: {"sub": "u"}
    assert p.authorization_url("s", "n1", "c").startswith("https://idp.example/auth?")
    token["id_token"] = signed(k_old, "old")
    assert p.exchange_code("c", "v", "n1")["sub"] == "acme:u"
    for bad, why in ((signed(k_old, "old", iss="https://evil"), "issuer"),
                     (signed(k_old, "old", aud="other"), "audience"),
                     (signed(k_old, "old", exp=int(_t.time()) - 3600), "expired"),
                     (signed(k_old, "old", nonce="n2"), "nonce")):
        token["id_token"] = bad
        with pytest.raises(PermissionError, match=why):
            p.exchange_code("c", "v", "n1")
    h, b, _ = signed(k_old, "old").split(".")
    token["id_token"] = f"{h}.{b}.{J.b64u(k_new.sign(f'{h}.{b}'.encode()))}"   # signed by a key not in JWKS
    with pytest.raises(PermissionError, match="signature"):
        p.exchange_code("c", "v", "n1")
    # rotation: the provider starts signing with "new"; the first miss refetches the JWKS
    jwks["keys"].append(k_new.public_jwk("new"))
    n_before = len(fetched)
    token["id_token"] = signed(k_new, "new")
    assert p.exchange_code("c", "v", "n1")["sub"] == "acme:u"
    assert len(fetched) == n_before + 1
    token["id_token"] = signed(k_new, "gone")
    with pytest.raises(PermissionError, match="not in the provider JWKS"):
        p.exchange_code("c", "v", "n1")
    # HS256 (a symmetric alg an attacker could forge with a public key) is refused outright
    token["id_token"] = J.encode({"iss": "https://idp.example", "aud": "client-1", "nonce": "n1"}, J.HMACSigner("x"))
    with pytest.raises(PermissionError, match="algorithm"):
        p.exchange_code("c", "v", "n1")


def test_auth_service_require_nonce_flag_reaches_providers():
    p = _FakeOIDC.make({"access_token": "at"}, {"sub": "u"})
    store = InMemoryDocumentStore()
    mgr = J.JWTManager(J.HMACSigner("k"))
    svc = AuthService(mgr, RoleStore(store), {"acme": p}, require_nonce=False)
    assert p.require_nonce is False
    st = svc.initiate_login("acme")["state"]
    assert svc.handle_callback("code", st)["user"]["user_id"] == "acme:u"


def test_es256_ladder_matches_double_and_add():
    import secrets as _s

    def naive(k, pt):
        R, Q = (0, 1, 0), (pt[0], pt[1], 1)
        while k:
            if k & 1:
                R = J._jadd(R, Q)
            Q = J._jdouble(Q)
            k >>= 1
        zi = pow(R[2], -1, J._P)
        return (R[0] * zi * zi % J._P, R[1] * zi * zi * zi % J._P)

    for k in (1, 2, 3, J._N - 1, _s.randbelow(J._N - 1) + 1):
        assert J._jmul(k, J._G) == naive(k, J._G)
    assert J._jmul(J._N, J._G) is None


def test_rsa_crt_fault_is_caught():
    key = J.RSAKey.generate(1024)
    key.dp ^= 1 << 5          # simulate a faulty half-exponentiation
    with pytest.raises(J.JWTError, match="self-check"):
        key.sign(b"payload")


def test_refresh_refuses_sessions_past_max_lifetime_and_denied_users():
    import time as _t
    store = InMemoryDocumentStore()
    mgr = J.JWTManager(J.HMACSigner("k"))
    svc = AuthService(mgr, RoleStore(store), {"mock": __import__(
        "copilot_for_consensus_amd.security.auth", fromlist=["MockIdentityProvider"]).MockIdentityProvider()},
        max_session_seconds=100)
    st = svc.initiate_login("mock")["state"]
    tok = svc.handle_callback("alice", st)["access_token"]
    new = svc.refresh(tok)["access_token"]
    assert J.decode_unverified(new)[1]["auth_time"] == J.decode_unverified(tok)[1]["auth_time"]   # kept, not reset
    old = mgr.mint_token("mock:alice", {"auth_time": int(_t.time()) - 1000})
    with pytest.raises(PermissionError, match="lifetime"):
        svc.refresh(old)
    svc.roles.deny("mock:alice")
    with pytest.raises(PermissionError, match="denied"):
        svc.refresh(tok)


def test_public_key_check_reads_jwk_and_rejects_mismatch():
    """A configured public key given as a JWK / JWKS is compared with the private key too (not only
    PEM): the matching key passes, another key or an unreadable value is refused."""
    import json

    from copilot_for_consensus_amd.security.jwt import ECKey, ECSigner, JWTError, RSAKey, RSASigner
    rk, other = RSAKey.generate(1024), RSAKey.generate(1024)
    RSASigner(rk, public_key=json.dumps(rk.public_jwk("k")))
    RSASigner(rk, public_key=json.dumps({"keys": [rk.public_jwk("k")]}))
    RSASigner(rk, public_key=J.rsa_public_pem(rk))
    with pytest.raises(JWTError):
        RSASigner(rk, public_key=json.dumps(other.public_jwk("k")))
    with pytest.raises(JWTError):
        RSASigner(rk, public_key="not a key")
    ek = ECKey.generate()
    ECSigner(ek, public_key=json.dumps(ek.public_jwk("e")))
    with pytest.raises(JWTError):
        ECSigner(ek, public_key=json.dumps(ECKey.generate().public_jwk("e")))
    with pytest.raises(JWTError):          # an RSA public key for an EC private key
        ECSigner(ek, public_key=json.dumps(rk.public_jwk("k")))
