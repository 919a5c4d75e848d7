"""Auth service routes (reference auth/main.py:115-1074): /providers /login /callback /refresh
POST /logout POST /token /userinfo /keys /.well-known/jwks.json /.well-known/public_key.pem
/admin/role-assignments/pending /admin/users/search GET/POST/DELETE /admin/users/{id}/roles
POST /admin/users/{id}/deny."""
from __future__ import annotations

from ..security.auth import AuthService, JWTMiddleware


def create_auth_app(svc: AuthService, cookie_secure: bool = False, token_exchange_secret: str | None = None):
    from fastapi import Cookie, Depends, FastAPI, Header, HTTPException, Query
    from fastapi.responses import JSONResponse, RedirectResponse

    app = FastAPI(title="copilot-for-consensus auth")
    admin = JWTMiddleware(verify_key=svc.jwt.signer, audience=svc.jwt.audience, required_roles=["admin"]).dependency()
    user = JWTMiddleware(verify_key=svc.jwt.signer, audience=svc.jwt.audience).dependency()

    @app.get("/health")
    def health():
        return {"status": "healthy", "service": "auth", "providers": sorted(svc.providers)}

    @app.get("/readyz")
    def readyz():
        return {"status": "ready"}

    @app.get("/providers")
    def providers():
        return {"providers": sorted(svc.providers)}

    @app.get("/login")
    def login(provider: str, aud: str | None = None, redirect: bool = False):
        try:
            r = svc.initiate_login(provider, aud)
        except KeyError as e:
            raise HTTPException(400, str(e))
        return RedirectResponse(r["authorization_url"]) if redirect else r

    @app.get("/callback")
    def callback(code: str, state: str, provider: str | None = None):
        try:
            r = svc.handle_callback(code, state)
        except PermissionError as e:
            raise HTTPException(401, str(e))
        resp = JSONResponse(r)
        # the cookie lives exactly as long as the token it carries
        resp.set_cookie("auth_token", r["access_token"], httponly=True, secure=cookie_secure, samesite="lax",
                        max_age=int(r["expires_in"]))
        return resp

    @app.get("/refresh")
    def refresh(authorization: str | None = Header(default=None), auth_token: str | None = Cookie(default=None)):
        """Re-mint a still-valid token with the user's CURRENT roles and the token's audience;
        the token comes from the Authorization header or the ``auth_token`` cookie."""
        tok = authorization[7:] if authorization and authorization.lower().startswith("bearer ") else auth_token
        if not tok:
            raise HTTPException(401, "No token found to refresh")
        if tok.count(".") != 2:
            raise HTTPException(400, "Malformed token")
        try:
            r = svc.refresh(tok)
        except Exception as e:
            raise HTTPException(401, str(e))
        resp = JSONResponse(r)
        resp.set_cookie("auth_token", r["access_token"], httponly=True, secure=cookie_secure, samesite="lax",
                        max_age=int(r["expires_in"]))
        return resp

    @app.post("/logout")
    def logout():
        resp = JSONResponse({"status": "logged out", "message": "auth_token cookie cleared"})
        resp.delete_cookie("auth_token", httponly=True, secure=cookie_secure, samesite="lax")
        return resp

    @app.post("/token")
    def token(body: dict):
        """Service-to-service token exchange guarded by a shared secret."""
        if not token_exchange_secret or body.get("secret") != token_exchange_secret:
            raise HTTPException(401, "invalid client credentials")
        roles = body.get("roles") or ["processor"]
        tok = svc.jwt.mint_token(body.get("subject", "service"), {"roles": roles}, audience=body.get("audience"))
        return {"access_token": tok, "token_type": "Bearer", "expires_in": svc.jwt.default_expiry}

    @app.get("/userinfo")
    def userinfo(claims: dict = Depends(user)):
        out = {k: claims.get(k) for k in ("sub", "email", "name", "provider", "aud", "exp")}
        out["roles"] = claims.get("roles", [])
        out["affiliations"] = claims.get("affiliations", [])
        return out

    @app.get("/keys")
    @app.get("/.well-known/jwks.json")
    def jwks():
        return svc.get_jwks()

    @app.get("/.well-known/public_key.pem")
    def public_key():
        k = svc.get_jwks()["keys"]
        if not k:
            raise HTTPException(404, "symmetric signer has no public key")
        return k[0]

    @app.get("/admin/role-assignments/pending")
    def pending(user_id: str | None = None, role: str | None = None, limit: int = Query(50, ge=1, le=100),
                skip: int = Query(0, ge=0), sort_by: str = "requested_at", sort_order: int = Query(-1, ge=-1, le=1),
                _admin: dict = Depends(admin)):
        page, total = svc.roles.pending(user_id=user_id, role=role, limit=limit, skip=skip, sort_by=sort_by,
                                        sort_order=sort_order)
        return {"assignments": page, "pending": page, "total": total, "limit": limit, "skip": skip}

    @app.get("/admin/users/search")
    def search(search_term: str | None = None, search_by: str = "email", q: str | None = None,
               _admin: dict = Depends(admin)):
        term = search_term if search_term is not None else q
        if not term:
            raise HTTPException(422, "search_term is required")
        if q is not None and search_term is None and search_by == "email":
            # the UI's free-text box: email or name
            users = svc.roles.search(term, "email")
            seen = {u["_id"] for u in users}
            users += [u for u in svc.roles.search(term, "name") if u["_id"] not in seen]
        else:
            try:
                users = svc.roles.search(term, search_by)
            except ValueError as e:
                raise HTTPException(400, str(e))
        return {"users": users, "count": len(users), "search_term": term, "search_by": search_by}

    @app.get("/admin/users/{user_id}/roles")
    def get_roles(user_id: str, _admin: dict = Depends(admin)):
        d = svc.roles.get(user_id)
        if d is None:
            raise HTTPException(404, f"User not found: {user_id}")
        return {"user_id": user_id, "email": d.get("email"), "name": d.get("name"), "roles": d.get("roles", []),
                "status": d.get("status")}

    def _roles_body(body: dict) -> list:
        roles = body.get("roles")
        if not isinstance(roles, list) or not roles:
            raise HTTPException(422, [{"loc": ["body", "roles"], "msg": "at least one role is required",
                                       "type": "too_short"}])
        return roles

    @app.post("/admin/users/{user_id}/roles")
    def assign(user_id: str, body: dict, claims: dict = Depends(admin)):
        try:
            return svc.roles.assign(user_id, _roles_body(body), admin_user_id=claims.get("sub"))
        except ValueError as e:
            raise HTTPException(400, str(e))

    @app.delete("/admin/users/{user_id}/roles")
    def revoke(user_id: str, body: dict, claims: dict = Depends(admin)):
        try:
            return svc.roles.revoke(user_id, _roles_body(body), admin_user_id=claims.get("sub"))
        except KeyError as e:
            raise HTTPException(404, str(e).strip("'"))
        except ValueError as e:
            raise HTTPException(400, str(e))

    @app.post("/admin/users/{user_id}/deny")
    def deny(user_id: str, claims: dict = Depends(admin)):
        try:
            return svc.roles.deny(user_id, admin_user_id=claims.get("sub"))
        except KeyError as e:
            raise HTTPException(404, str(e).strip("'"))
        except ValueError as e:   # not pending (already approved or denied)
            raise HTTPException(409, str(e))

    return app
