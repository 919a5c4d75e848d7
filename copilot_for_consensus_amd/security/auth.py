"""Authentication: OIDC identity providers (PKCE + nonce), role store, service JWT middleware.

Reference: adapters/copilot_auth (OIDCProvider oidc_provider.py:23 with PKCE :360; GitHub / Google /
Microsoft / Mock providers; JWTMiddleware middleware.py:52 with JWKS fetch :122-270 and role check
:424), auth/app/service.py:171 (initiate_login :398, handle_callback :471, validate_token :583,
get_jwks :625) and auth/app/role_store.py:28.
"""
from __future__ import annotations

import base64
import hashlib
import json
import secrets
import threading
import time
import urllib.parse
import urllib.request
from abc import ABC, abstractmethod
from datetime import datetime, timezone
from typing import Any

from .jwt import ECKey, JWTError, JWTManager, RSAKey, decode, decode_unverified


def pkce_pair() -> tuple[str, str]:
    verifier = base64.urlsafe_b64encode(secrets.token_bytes(32)).rstrip(b"=").decode()
    challenge = base64.urlsafe_b64encode(hashlib.sha256(verifier.encode()).digest()).rstrip(b"=").decode()
    return verifier, challenge


class IdentityProvider(ABC):
    name = "base"

    @abstractmethod
    def authorization_url(self, state: str, nonce: str, code_challenge: str) -> str: ...

    @abstractmethod
    def exchange_code(self, code: str, code_verifier: str, nonce: str) -> dict:
        """-> user info {sub, email, name, provider}."""


class OIDCProvider(IdentityProvider):
    """OAuth2 / OpenID Connect code flow with PKCE.  With a ``discovery_url`` (or an ``issuer``,
    whose ``/.well-known/openid-configuration`` is used) the endpoints, issuer and JWKS URI come
    from discovery (reference oidc_provider.py:72-96) and every id_token is verified: RS256 / ES256
    signature against the provider's JWKS (re-fetched once on an unknown ``kid``: key rotation),
    ``iss``, ``aud`` = client_id, ``exp`` / ``nbf`` with leeway and ``nonce``
    (oidc_provider.py:312-355).  Plain OAuth providers (GitHub) have no id_token."""

    JWKS_TTL = 3600.0

    def __init__(self, name: str, client_id: str, client_secret: str, redirect_uri: str,
                 authorize_endpoint: str | None = None, token_endpoint: str | None = None,
                 userinfo_endpoint: str | None = None, scope: str = "openid email profile",
                 discovery_url: str | None = None, issuer: str | None = None, jwks_uri: str | None = None,
                 leeway: int = 60):
        self.name = name
        self.client_id, self.client_secret, self.redirect_uri = client_id, client_secret, redirect_uri
        self.authorize_endpoint, self.token_endpoint = authorize_endpoint, token_endpoint
        self.userinfo_endpoint, self.scope = userinfo_endpoint, scope
        if discovery_url is None and issuer:
            discovery_url = issuer.rstrip("/") + "/.well-known/openid-configuration"
        self.discovery_url, self.issuer, self.jwks_uri, self.leeway = discovery_url, issuer, jwks_uri, leeway
        self._discovered = False
        self._jwks: dict | None = None
        self._jwks_at = 0.0
        self._lock = threading.Lock()

    def _fetch_json(self, url: str) -> dict:
        req = urllib.request.Request(url, headers={"Accept": "application/json"})
        return json.loads(urllib.request.urlopen(req, timeout=10).read())

    def discover(self) -> None:
        """Endpoints, issuer and jwks_uri from the discovery document (explicit arguments win)."""
        if self._discovered or not self.discovery_url:
            return
        try:
            doc = self._fetch_json(self.discovery_url)
        except (OSError, ValueError) as e:
            raise PermissionError(f"{self.name}: OIDC discovery failed: {e}") from e
        self.authorize_endpoint = self.authorize_endpoint or doc.get("authorization_endpoint")
        self.token_endpoint = self.token_endpoint or doc.get("token_endpoint")
        self.userinfo_endpoint = self.userinfo_endpoint or doc.get("userinfo_endpoint")
        self.jwks_uri = self.jwks_uri or doc.get("jwks_uri")
        self.issuer = self.issuer or doc.get("issuer")
        if not (self.authorize_endpoint and self.token_endpoint):
            raise PermissionError(f"{self.name}: discovery document lacks authorization/token endpoints")
        self._discovered = True

    def _signing_key(self, header: dict):
        """The JWKS key for this token's kid (one refresh on a miss or after JWKS_TTL)."""
        for attempt in (0, 1):
            with self._lock:
                stale = self._jwks is None or time.time() - self._jwks_at > self.JWKS_TTL or attempt == 1
                if stale:
                    try:
                        self._jwks, self._jwks_at = self._fetch_json(self.jwks_uri), time.time()
                    except (OSError, ValueError) as e:
                        raise PermissionError(f"{self.name}: JWKS fetch failed: {e}") from e
                keys = [k for k in self._jwks.get("keys", []) if k.get("use", "sig") == "sig"]
            kid = header.get("kid")
            match = [k for k in keys if k.get("kid") == kid] if kid else (keys if len(keys) == 1 else [])
            if match:
                jwk = match[0]
                return ECKey.from_jwk(jwk) if jwk.get("kty") == "EC" else RSAKey.from_jwk(jwk)
            if stale:
                break
        raise PermissionError(f"{self.name}: id_token key {header.get('kid')!r} not in the provider JWKS")

    def _expected_issuer(self, claims: dict) -> str | None:
        iss = self.issuer
        if iss and "{tenantid}" in iss:   # Microsoft multi-tenant discovery documents template the tenant
            iss = iss.replace("{tenantid}", str(claims.get("tid", "")))
        return iss

    def verify_id_token(self, id_token: str, nonce: str) -> dict:
        """Verified id_token claims (signature, iss, aud, exp/nbf, nonce); raises PermissionError."""
        self.discover()
        try:
            header, claims = decode_unverified(id_token)
        except JWTError as e:
            raise PermissionError("malformed id_token") from e
        if header.get("alg") not in ("RS256", "ES256"):
            raise PermissionError(f"id_token algorithm {header.get('alg')!r} not accepted")
        if self.jwks_uri:
            try:
                claims = decode(id_token, self._signing_key(header), audience=self.client_id,
                                issuer=self._expected_issuer(claims), leeway=self.leeway)
            except JWTError as e:
                raise PermissionError(f"id_token rejected: {e}") from e
        else:
            # no JWKS published: the token came straight from the token endpoint over TLS (OIDC Core
            # 3.1.3.7); the registered claims are still checked
            now = time.time()
            if "exp" in claims and now > claims["exp"] + self.leeway:
                raise PermissionError("id_token expired")
            aud = claims.get("aud")
            if self.client_id not in (aud if isinstance(aud, list) else [aud]):
                raise PermissionError("id_token audience mismatch")
            want = self._expected_issuer(claims)
            if want and claims.get("iss") != want:
                raise PermissionError("id_token issuer mismatch")
        if claims.get("nonce") != nonce:
            raise PermissionError("id_token nonce mismatch")
        return claims

    def authorization_url(self, state, nonce, code_challenge):
        self.discover()
        q = {"response_type": "code", "client_id": self.client_id, "redirect_uri": self.redirect_uri,
             "scope": self.scope, "state": state, "nonce": nonce, "code_challenge": code_challenge,
             "code_challenge_method": "S256"}
        return f"{self.authorize_endpoint}?{urllib.parse.urlencode(q)}"

    def _post(self, url, data):
        req = urllib.request.Request(url, data=urllib.parse.urlencode(data).encode(),
                                     headers={"Accept": "application/json"})
        return json.loads(urllib.request.urlopen(req, timeout=15).read())

    def _get(self, url, token):
        req = urllib.request.Request(url, headers={"Authorization": f"Bearer {token}", "Accept": "application/json"})
        return json.loads(urllib.request.urlopen(req, timeout=15).read())

    require_nonce = True

    def exchange_code(self, code, code_verifier, nonce):
        self.discover()
        tok = self._post(self.token_endpoint, {"grant_type": "authorization_code", "code": code,
                                               "redirect_uri": self.redirect_uri, "client_id": self.client_id,
                                               "client_secret": self.client_secret, "code_verifier": code_verifier})
        if "access_token" not in tok:
            raise PermissionError(f"token endpoint refused the code: {tok.get('error', 'no access_token')}")
        id_token = tok.get("id_token")
        if id_token:
            self.verify_id_token(id_token, nonce)
        elif self.require_nonce and "openid" in self.scope.split():
            # an OpenID provider must return an id_token carrying our nonce (plain OAuth providers
            # such as GitHub do not request the openid scope and have no nonce to check)
            raise PermissionError("OpenID provider returned no id_token to check the nonce against")
        info = self._get(self.userinfo_endpoint, tok["access_token"])
        subject = info.get("sub") or info.get("id")
        if subject in (None, ""):
            raise PermissionError("userinfo has no subject (sub / id)")
        return {"sub": f"{self.name}:{subject}", "email": info.get("email"),
                "name": info.get("name") or info.get("login"), "provider": self.name}


def github_provider(github_client_id, github_client_secret, github_redirect_uri=None,
                    github_api_base_url="https://api.github.com", **_):
    return OIDCProvider("github", github_client_id, github_client_secret, github_redirect_uri or "",
                        "https://github.com/login/oauth/authorize", "https://github.com/login/oauth/access_token",
                        f"{github_api_base_url}/user", scope="read:user user:email")


def google_provider(google_client_id, google_client_secret, google_redirect_uri=None, **_):
    return OIDCProvider("google", google_client_id, google_client_secret, google_redirect_uri or "",
                        issuer="https://accounts.google.com")


def microsoft_provider(microsoft_client_id, microsoft_client_secret, microsoft_redirect_uri=None,
                       microsoft_tenant="common", **_):
    return OIDCProvider("microsoft", microsoft_client_id, microsoft_client_secret, microsoft_redirect_uri or "",
                        discovery_url=f"https://login.microsoftonline.com/{microsoft_tenant}/v2.0/"
                                      ".well-known/openid-configuration")


def datatracker_provider(datatracker_client_id, datatracker_client_secret, datatracker_redirect_uri=None,
                         datatracker_issuer="https://auth.ietf.org/api/openid", **_):
    """IETF Datatracker login through its OpenID Connect provider (the reference ships only a
    scaffold that raises NotImplementedError, datatracker_provider.py:14)."""
    return OIDCProvider("datatracker", datatracker_client_id, datatracker_client_secret,
                        datatracker_redirect_uri or "", scope="openid profile email roles",
                        issuer=datatracker_issuer.rstrip("/"))


class MockIdentityProvider(IdentityProvider):
    """Deterministic provider for tests/dev (reference mock_provider.py:15): any code logs in the
    user whose id is the code."""
    name = "mock"

    def authorization_url(self, state, nonce, code_challenge):
        return f"/auth/callback?provider=mock&state={state}&code=mock-user"

    def exchange_code(self, code, code_verifier, nonce):
        return {"sub": f"mock:{code}", "email": f"{code}@example.com", "name": code, "provider": "mock"}


class RoleStore:
    """user -> roles with pending approvals (auth/app/role_store.py:28), persisted in a collection.

    Semantics of the reference: a new user is auto-promoted to admin + reader only when that is
    enabled AND no admin exists yet; otherwise the configured auto-approve roles, otherwise
    ``pending``.  Admin operations validate role names against ``VALID_ROLES``; assigning to an
    unknown user creates the record; deny applies to pending requests only."""

    VALID_ROLES = frozenset({"admin", "contributor", "reviewer", "reader"})
    SEARCH_FIELDS = ("user_id", "email", "name")

    def __init__(self, document_store, collection: str = "user_roles", auto_approve_roles: list[str] | None = None,
                 first_user_auto_promotion: bool = False):
        self.store, self.coll = document_store, collection
        self.auto_roles = [r for r in (auto_approve_roles or []) if r]
        self.first_user_admin = first_user_auto_promotion
        self._lock = threading.Lock()

    @staticmethod
    def _now() -> str:
        return datetime.now(timezone.utc).isoformat()

    def _check_roles(self, roles) -> list[str]:
        if not isinstance(roles, (list, tuple)) or not all(isinstance(r, str) for r in roles):
            raise ValueError("roles must be a list of role names")
        bad = [r for r in roles if r not in self.VALID_ROLES]
        if bad:
            raise ValueError(f"Invalid roles: {', '.join(bad)}. Valid roles are: {', '.join(sorted(self.VALID_ROLES))}")
        return list(roles)

    def get(self, user_id: str) -> dict | None:
        return self.store.get_document(self.coll, user_id)

    def find_by_role(self, role: str) -> list[dict]:
        return self.store.query_documents(self.coll, {"roles": role, "status": {"$ne": "denied"}}, limit=1 << 30)

    def ensure_user(self, user: dict) -> dict:
        with self._lock:
            doc = self.get(user["sub"])
            if doc is None:
                roles, status = [], "pending"
                if self.first_user_admin and not self.find_by_role("admin"):
                    roles, status = ["admin", "reader"], "approved"
                elif self.auto_roles:
                    roles, status = sorted(set(self.auto_roles)), "approved"
                now = self._now()
                doc = {"_id": user["sub"], "user_id": user["sub"], "email": user.get("email"), "name": user.get("name"),
                       "provider": user.get("provider"), "roles": roles, "status": status, "created_at": now,
                       "requested_at": now, "updated_at": now}
                self.store.insert_document(self.coll, doc)
            return doc

    def roles(self, user_id: str) -> list[str]:
        d = self.get(user_id)
        return list(d.get("roles", [])) if d and d.get("status") != "denied" else []

    def assign(self, user_id: str, roles: list[str], admin_user_id: str | None = None) -> dict:
        roles = self._check_roles(roles)
        now = self._now()
        with self._lock:
            d = self.get(user_id)
            patch = {"status": "approved", "updated_at": now, "approved_by": admin_user_id, "approved_at": now}
            if d is None:   # assigning to a user who never logged in creates the record
                self.store.insert_document(self.coll, {"_id": user_id, "user_id": user_id, "roles": sorted(set(roles)),
                                                       "created_at": now, **patch})
            else:
                self.store.update_document(self.coll, user_id,
                                           {"roles": sorted(set(d.get("roles", [])) | set(roles)), **patch})
            return self.get(user_id)

    def revoke(self, user_id: str, roles: list[str], admin_user_id: str | None = None) -> dict:
        roles = self._check_roles(roles)
        with self._lock:
            d = self.get(user_id)
            if d is None:
                raise KeyError(f"User record not found: {user_id}")
            keep = [r for r in d.get("roles", []) if r not in roles]
            self.store.update_document(self.coll, user_id, {"roles": keep, "updated_at": self._now(),
                                                            "last_modified_by": admin_user_id})
            return self.get(user_id)

    def deny(self, user_id: str, admin_user_id: str | None = None) -> dict:
        """Deny a PENDING request: KeyError if unknown, ValueError if not pending."""
        with self._lock:
            d = self.get(user_id)
            if d is None:
                raise KeyError(f"User record not found: {user_id}")
            if d.get("status", "pending") != "pending":
                raise ValueError(f"Cannot deny: user status is '{d.get('status')}', expected 'pending'")
            now = self._now()
            self.store.update_document(self.coll, user_id, {"status": "denied", "roles": [], "denied_by": admin_user_id,
                                                            "denied_at": now, "updated_at": now})
            return self.get(user_id)

    def pending(self, user_id: str | None = None, role: str | None = None, limit: int = 50, skip: int = 0,
                sort_by: str = "requested_at", sort_order: int = -1) -> tuple[list[dict], int]:
        """Pending requests filtered by user / role, sorted and paged -> (page, total)."""
        q: dict = {"status": "pending"}
        if user_id:
            q["user_id"] = user_id
        if role:
            q["roles"] = role
        total = self.store.count_documents(self.coll, q)
        page = self.store.query_documents(self.coll, q, limit=limit, skip=skip, sort_by=sort_by,
                                          sort_order="desc" if sort_order == -1 else "asc")
        return page, total

    def search(self, term: str, by: str = "email") -> list[dict]:
        """user_id: exact match; email / name: case-insensitive substring (records missing the
        field never match)."""
        if by not in self.SEARCH_FIELDS:
            raise ValueError(f"Invalid search_by field: {by}. Must be one of {', '.join(self.SEARCH_FIELDS)}")
        if by == "user_id":
            return self.store.query_documents(self.coll, {"user_id": term}, limit=1 << 30)
        t = term.lower()
        return [u for u in self.store.query_documents(self.coll, {}, limit=1 << 30)
                if isinstance(u.get(by), str) and t in u[by].lower()]


class JWTMiddleware:
    """Bearer-token verification + role check for the service APIs (middleware.py:52,424).

    ``verify_key`` is the auth service's signer (in-process) or a JWKS dict fetched from
    ``{auth_service_url}/keys`` (cached, refreshed on unknown kid)."""

    def __init__(self, verify_key=None, auth_service_url: str | None = None, audience: str = "copilot-for-consensus",
                 required_roles: list[str] | None = None, public_paths: tuple[str, ...] = ("/health", "/readyz")):
        self.verify_key, self.auth_url = verify_key, auth_service_url
        self.audience, self.required_roles = audience, set(required_roles or [])
        self.public_paths = public_paths
        self._jwks: dict | None = None
        self._jwks_at = 0.0

    def _key(self):
        if self.verify_key is not None:
            return self.verify_key
        if self._jwks is None or time.time() - self._jwks_at > 300:
            with urllib.request.urlopen(f"{self.auth_url}/keys", timeout=10) as r:
                self._jwks = json.loads(r.read())
            self._jwks_at = time.time()
        return self._jwks

    def verify(self, authorization: str | None) -> dict:
        if not authorization or not authorization.lower().startswith("bearer "):
            raise PermissionError("missing bearer token")
        try:
            claims = decode(authorization.split(" ", 1)[1], self._key(), audience=self.audience)
        except JWTError as e:
            raise PermissionError(str(e)) from e
        if self.required_roles and not (self.required_roles & set(claims.get("roles", []))):
            raise LookupError("insufficient role")
        return claims

    def dependency(self):
        from fastapi import Cookie, Header, HTTPException

        def dep(authorization: str | None = Header(default=None),
                auth_token: str | None = Cookie(default=None)) -> dict:
            # Authorization header first, then the httpOnly ``auth_token`` cookie the UI carries
            # (reference middleware.py:480-511)
            if not (authorization and authorization.lower().startswith("bearer ")) and auth_token:
                authorization = f"Bearer {auth_token}"
            try:
                return self.verify(authorization)
            except PermissionError as e:
                raise HTTPException(401, str(e))
            except LookupError as e:
                raise HTTPException(403, str(e))
        return dep


class AuthService:
    """Login flow state machine + token minting + role administration."""

    def __init__(self, jwt_manager: JWTManager, role_store: RoleStore, providers: dict[str, IdentityProvider],
                 require_pkce: bool = True, require_nonce: bool = True, state_ttl: int = 600,
                 max_session_seconds: int = 86400):
        self.jwt, self.roles, self.providers = jwt_manager, role_store, providers
        # a refresh keeps the login's auth_time; past this lifetime the user must log in again at the
        # provider (so a stolen token cannot be renewed forever and a revocation there takes effect)
        self.max_session_seconds = int(max_session_seconds)
        self.require_pkce, self.require_nonce = require_pkce, require_nonce
        for p in providers.values():   # the nonce is checked inside OIDCProvider.exchange_code
            if isinstance(p, OIDCProvider):
                p.require_nonce = require_nonce
        self._pending: dict[str, dict[str, Any]] = {}
        self.state_ttl = state_ttl
        self._lock = threading.Lock()

    def initiate_login(self, provider: str, audience: str | None = None) -> dict:
        p = self.providers.get(provider)
        if p is None:
            raise KeyError(f"unknown provider {provider}")
        state, nonce = secrets.token_urlsafe(24), secrets.token_urlsafe(24)
        verifier, challenge = pkce_pair()
        with self._lock:
            now = time.time()
            self._pending = {k: v for k, v in self._pending.items() if now - v["t"] < self.state_ttl}
            self._pending[state] = {"provider": provider, "nonce": nonce, "verifier": verifier, "t": now,
                                    "audience": audience}
        return {"authorization_url": p.authorization_url(state, nonce, challenge), "state": state}

    def handle_callback(self, code: str, state: str) -> dict:
        with self._lock:
            st = self._pending.pop(state, None)
        if st is None or time.time() - st["t"] > self.state_ttl:
            raise PermissionError("invalid or expired state")
        user = self.providers[st["provider"]].exchange_code(code, st["verifier"], st["nonce"])
        doc = self.roles.ensure_user(user)
        token = self.jwt.mint_token(user["sub"], {"email": user.get("email"), "name": user.get("name"),
                                                  "roles": self.roles.roles(user["sub"]),
                                                  "provider": user.get("provider"), "auth_time": int(time.time())},
                                    audience=st.get("audience"))
        return {"access_token": token, "token_type": "Bearer", "expires_in": self.jwt.default_expiry,
                "user": {k: doc.get(k) for k in ("user_id", "email", "name", "roles", "status")}}

    def validate_token(self, token: str, audience: str | None = None) -> dict:
        return self.jwt.validate_token(token, audience)

    def refresh(self, token: str) -> dict:
        """Signature and expiry are checked against the audience the token was minted for, and
        the new token keeps that audience (reference main.py refresh: audience preserved)."""
        from .jwt import decode_unverified
        _, unverified = decode_unverified(token)
        aud = unverified.get("aud")
        aud = aud[0] if isinstance(aud, list) and aud else aud
        claims = self.jwt.validate_token(token, audience=aud if isinstance(aud, str) else None)
        sub = claims.get("sub")
        if not isinstance(sub, str) or not sub:
            raise PermissionError("Missing or invalid 'sub' claim in token")
        auth_time = claims.get("auth_time", claims.get("iat"))
        if not isinstance(auth_time, (int, float)) or time.time() - auth_time > self.max_session_seconds:
            raise PermissionError("session older than the maximum lifetime: log in again")
        if self.roles.get(sub) is not None and self.roles.get(sub).get("status") == "denied":
            raise PermissionError("user access has been denied")
        new = self.jwt.mint_token(sub, {k: claims.get(k) for k in ("email", "name", "provider")} |
                                  {"roles": self.roles.roles(sub), "auth_time": int(auth_time)},
                                  audience=aud if isinstance(aud, str) else None)
        return {"access_token": new, "token_type": "Bearer", "expires_in": self.jwt.default_expiry}

    def get_jwks(self) -> dict:
        return self.jwt.get_jwks()
