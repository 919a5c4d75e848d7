"""Auth service admin and token routes with the reference's semantics (auth/tests/test_admin_endpoints.py,
test_role_store_admin.py, test_auto_promotion.py, test_userinfo*.py, test_refresh*.py,
test_cookie*.py): role validation, merge / dedupe, assignment creating unknown users, revoke of
absent roles, deny only from pending (409 otherwise, 404 unknown), pending list filters / paging /
sorting, search by field, header-over-cookie precedence, cookie lifetime, refresh keeping the
audience and picking up current roles, auto-promotion only while no admin exists."""
from __future__ import annotations

import pytest
from fastapi.testclient import TestClient

from copilot_for_consensus_amd.security import jwt as J
from copilot_for_consensus_amd.security.auth import AuthService, MockIdentityProvider, RoleStore
from copilot_for_consensus_amd.services.auth import create_auth_app
from copilot_for_consensus_amd.storage.document_store import InMemoryDocumentStore


def make(first_admin=True, auto_roles=None):
    store = InMemoryDocumentStore()
    roles = RoleStore(store, first_user_auto_promotion=first_admin, auto_approve_roles=auto_roles)
    mgr = J.JWTManager(J.HMACSigner("k"), issuer="copilot-auth", audience="copilot-for-consensus", default_expiry=900)
    svc = AuthService(mgr, roles, {"mock": MockIdentityProvider()})
    return svc, TestClient(create_auth_app(svc))


def login(c, code, aud=None):
    start = c.get("/login", params={"provider": "mock", **({"aud": aud} if aud else {})}).json()
    r = c.get("/callback", params={"code": code, "state": start["state"]})
    assert r.status_code == 200, r.text
    c.cookies.clear()
    return r


def H(tok):
    return {"Authorization": f"Bearer {tok}"}


@pytest.fixture
def env():
    svc, c = make()
    admin = login(c, "alice").json()["access_token"]
    return svc, c, admin


# ------------------------------------------------------------------ role store semantics
def test_auto_promotion_only_while_no_admin_exists():
    svc, c = make()
    assert login(c, "a").json()["user"]["roles"] == ["admin", "reader"]
    assert login(c, "b").json()["user"]["status"] == "pending"
    # the admin's record is deleted: the next NEW user is promoted again, existing users are not
    svc.roles.store.delete_document("user_roles", "mock:a")
    assert login(c, "b").json()["user"]["status"] == "pending"
    assert login(c, "c").json()["user"]["roles"] == ["admin", "reader"]


def test_auto_promotion_disabled_by_default_falls_back_to_auto_approve():
    _, c = make(first_admin=False)
    assert login(c, "a").json()["user"]["status"] == "pending"
    _, c = make(first_admin=False, auto_roles=["reader", ""])
    u = login(c, "a").json()["user"]
    assert u["roles"] == ["reader"] and u["status"] == "approved"


def test_denied_user_gets_no_roles_in_new_tokens(env):
    svc, c, admin = env
    login(c, "mallory")
    assert c.post("/admin/users/mock:mallory/deny", headers=H(admin)).json()["status"] == "denied"
    tok = login(c, "mallory").json()["access_token"]
    assert svc.validate_token(tok)["roles"] == []


# ------------------------------------------------------------------ assign / revoke / deny
def test_assign_merges_dedupes_and_records_admin(env):
    svc, c, admin = env
    login(c, "bob")
    r = c.post("/admin/users/mock:bob/roles", json={"roles": ["reader", "reader"]}, headers=H(admin)).json()
    assert r["roles"] == ["reader"] and r["status"] == "approved" and r["approved_by"] == "mock:alice"
    r = c.post("/admin/users/mock:bob/roles", json={"roles": ["contributor", "reader"]}, headers=H(admin)).json()
    assert r["roles"] == ["contributor", "reader"]
    assert "_id" in r and r["_id"] == "mock:bob"


@pytest.mark.parametrize("body,code", [({"roles": []}, 422), ({}, 422), ({"roles": "reader"}, 422),
                                       ({"roles": ["superuser"]}, 400), ({"roles": ["reader", "root"]}, 400)])
def test_assign_validation(env, body, code):
    _, c, admin = env
    login(c, "bob")
    assert c.post("/admin/users/mock:bob/roles", json=body, headers=H(admin)).status_code == code


def test_assign_to_unknown_user_creates_record(env):
    _, c, admin = env
    r = c.post("/admin/users/github:999/roles", json={"roles": ["reviewer"]}, headers=H(admin))
    assert r.status_code == 200 and r.json()["user_id"] == "github:999" and r.json()["status"] == "approved"
    assert c.get("/admin/users/github:999/roles", headers=H(admin)).json()["roles"] == ["reviewer"]


def test_revoke(env):
    _, c, admin = env
    login(c, "bob")
    c.post("/admin/users/mock:bob/roles", json={"roles": ["reader", "contributor"]}, headers=H(admin))
    r = c.request("DELETE", "/admin/users/mock:bob/roles", json={"roles": ["admin"]}, headers=H(admin))
    assert r.json()["roles"] == ["contributor", "reader"]          # absent role: unchanged
    r = c.request("DELETE", "/admin/users/mock:bob/roles", json={"roles": ["contributor", "reader"]},
                  headers=H(admin))
    assert r.json()["roles"] == [] and r.json()["last_modified_by"] == "mock:alice"
    assert c.request("DELETE", "/admin/users/mock:bob/roles", json={"roles": ["wizard"]},
                     headers=H(admin)).status_code == 400
    assert c.request("DELETE", "/admin/users/ghost/roles", json={"roles": ["reader"]},
                     headers=H(admin)).status_code == 404


def test_deny_rules(env):
    _, c, admin = env
    login(c, "bob")
    r = c.post("/admin/users/mock:bob/deny", headers=H(admin))
    assert r.status_code == 200 and r.json()["status"] == "denied" and r.json()["roles"] == []
    assert c.post("/admin/users/mock:bob/deny", headers=H(admin)).status_code == 409     # already denied
    assert c.post("/admin/users/mock:alice/deny", headers=H(admin)).status_code == 409   # approved
    assert c.post("/admin/users/ghost/deny", headers=H(admin)).status_code == 404


# ------------------------------------------------------------------ pending list + search
def test_pending_filters_paging_and_sorting(env):
    svc, c, admin = env
    for u in ("u1", "u2", "u3", "u4"):
        login(c, u)
    svc.roles.store.update_document("user_roles", "mock:u2", {"roles": ["contributor"]})  # a requested role
    r = c.get("/admin/role-assignments/pending", headers=H(admin)).json()
    assert r["total"] == 4 and r["limit"] == 50 and r["skip"] == 0
    assert [a["user_id"] for a in r["assignments"]] == ["mock:u4", "mock:u3", "mock:u2", "mock:u1"]  # newest first
    r = c.get("/admin/role-assignments/pending", params={"sort_order": 1, "limit": 2, "skip": 1}, headers=H(admin))
    assert [a["user_id"] for a in r.json()["assignments"]] == ["mock:u2", "mock:u3"] and r.json()["total"] == 4
    r = c.get("/admin/role-assignments/pending", params={"user_id": "mock:u3"}, headers=H(admin)).json()
    assert [a["user_id"] for a in r["assignments"]] == ["mock:u3"] and r["total"] == 1
    r = c.get("/admin/role-assignments/pending", params={"role": "contributor"}, headers=H(admin)).json()
    assert [a["user_id"] for a in r["assignments"]] == ["mock:u2"]
    for bad in ({"limit": 0}, {"limit": 101}, {"skip": -1}, {"sort_order": 2}):
        assert c.get("/admin/role-assignments/pending", params=bad, headers=H(admin)).status_code == 422


def test_search_by_field(env):
    svc, c, admin = env
    login(c, "Bobby")
    svc.roles.store.insert_document("user_roles", {"_id": "x:noemail", "user_id": "x:noemail", "name": "Bob",
                                                   "roles": [], "status": "pending"})
    s = lambda **p: c.get("/admin/users/search", params=p, headers=H(admin))  # noqa: E731
    assert [u["user_id"] for u in s(search_term="BOBBY@EXAMPLE").json()["users"]] == ["mock:Bobby"]
    assert sorted(u["user_id"] for u in s(search_term="bob", search_by="name").json()["users"]) == \
        ["mock:Bobby", "x:noemail"]
    assert [u["user_id"] for u in s(search_term="mock:Bobby", search_by="user_id").json()["users"]] == ["mock:Bobby"]
    assert s(search_term="mock:Bob", search_by="user_id").json()["users"] == []        # exact match only
    assert s(search_term="zzz").json()["users"] == []
    assert s(search_term="bob", search_by="phone").status_code == 400
    assert s().status_code == 422


# ------------------------------------------------------------------ tokens, cookies, userinfo
def test_admin_routes_require_admin(env):
    _, c, admin = env
    user = login(c, "bob").json()["access_token"]
    assert c.get("/admin/role-assignments/pending").status_code == 401
    assert c.get("/admin/role-assignments/pending", headers=H(user)).status_code == 403
    assert c.get("/admin/role-assignments/pending", headers=H("garbage")).status_code == 401
    assert c.get("/admin/role-assignments/pending", cookies={"auth_token": admin}).status_code == 200


def test_header_takes_precedence_over_cookie(env):
    _, c, admin = env
    user = login(c, "bob").json()["access_token"]
    r = c.get("/admin/role-assignments/pending", headers=H(user), cookies={"auth_token": admin})
    assert r.status_code == 403
    assert c.get("/userinfo", headers=H(user), cookies={"auth_token": admin}).json()["sub"] == "mock:bob"


def test_userinfo_contents_and_invalid_tokens(env):
    _, c, admin = env
    info = c.get("/userinfo", headers=H(admin)).json()
    assert info["sub"] == "mock:alice" and info["email"] == "alice@example.com"
    assert info["roles"] == ["admin", "reader"] and info["aud"] == "copilot-for-consensus"
    assert isinstance(info["exp"], int) and info["affiliations"] == []
    assert c.get("/userinfo", cookies={"auth_token": admin}).json()["sub"] == "mock:alice"
    assert c.get("/userinfo", cookies={"auth_token": "not-a-jwt"}).status_code == 401
    assert c.get("/userinfo", headers=H("a.b.c")).status_code == 401
    assert c.get("/userinfo").status_code == 401


def test_callback_cookie_lifetime_and_logout():
    _, c = make()
    start = c.get("/login", params={"provider": "mock"}).json()
    r = c.get("/callback", params={"code": "alice", "state": start["state"]})
    cookie = r.headers["set-cookie"]
    assert "auth_token=" in cookie and "HttpOnly" in cookie and "Max-Age=900" in cookie
    out = c.post("/logout")
    assert out.status_code == 200 and 'auth_token=""' in out.headers["set-cookie"]
    assert "Max-Age=0" in out.headers["set-cookie"]


def test_secure_cookie_flag():
    store = InMemoryDocumentStore()
    svc = AuthService(J.JWTManager(J.HMACSigner("k")), RoleStore(store), {"mock": MockIdentityProvider()})
    c = TestClient(create_auth_app(svc, cookie_secure=True))
    start = c.get("/login", params={"provider": "mock"}).json()
    assert "Secure" in c.get("/callback", params={"code": "a", "state": start["state"]}).headers["set-cookie"]


def test_refresh_keeps_audience_and_picks_up_current_roles():
    svc, c = make()
    login(c, "alice")
    bob = login(c, "bob", aud="reporting-ui").json()["access_token"]
    assert svc.jwt.validate_token(bob, audience="reporting-ui")["roles"] == []
    admin = svc.jwt.mint_token("mock:alice", {"roles": ["admin"]})
    c.post("/admin/users/mock:bob/roles", json={"roles": ["reader"]}, headers=H(admin))
    new = c.get("/refresh", headers=H(bob))
    assert new.status_code == 200 and "auth_token=" in new.headers["set-cookie"]
    claims = svc.jwt.validate_token(new.json()["access_token"], audience="reporting-ui")
    assert claims["roles"] == ["reader"] and claims["aud"] == "reporting-ui" and claims["sub"] == "mock:bob"
    assert c.get("/refresh", cookies={"auth_token": bob}).status_code == 200


@pytest.mark.parametrize("hdr,code", [(None, 401), ("Bearer not-a-token", 400), ("Bearer a.b.c", 401)])
def test_refresh_errors(hdr, code):
    _, c = make()
    assert c.get("/refresh", headers={"Authorization": hdr} if hdr else {}).status_code == code


def test_refresh_rejects_expired_and_foreign_tokens():
    svc, c = make()
    expired = svc.jwt.mint_token("mock:x", {}, expires_in=-1000)
    assert c.get("/refresh", headers=H(expired)).status_code == 401
    foreign = J.JWTManager(J.HMACSigner("other-key"), issuer="copilot-auth").mint_token("mock:x")
    assert c.get("/refresh", headers=H(foreign)).status_code == 401
    nosub = J.encode({"iss": svc.jwt.issuer, "aud": svc.jwt.audience, "exp": 2 ** 31}, svc.jwt.signer)
    assert c.get("/refresh", headers=H(nosub)).status_code == 401


def test_providers_and_unknown_provider_login():
    _, c = make()
    assert c.get("/providers").json()["providers"] == ["mock"]
    r = c.get("/login", params={"provider": "google"})
    assert r.status_code == 400 and "google" in r.text
