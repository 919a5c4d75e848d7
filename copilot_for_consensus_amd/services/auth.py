"""Auth service routes (reference auth/main.py:115-1074): /providers /login /callback /refresh
POST /logout POST /token /userinfo /keys /.well-known/jwks.json /.well-known/public_key.pem
/admin/role-assignments/pending /admin/users/search GET/POST/DELETE /admin/users/{id}/roles
POST /admin/users/{id}/deny."""
from __future__ import annotations

from ..security.auth import AuthService, JWTMiddleware


def create_auth_app(svc: AuthService, cookie_secure: bool = False, token_exchange_secret: str | None = None):
    from fastapi import Depends, FastAPI, Header, HTTPException
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
        resp.set_cookie("auth_token", r["access_token"], httponly=True, secure=cookie_secure, samesite="lax")
        return resp

    @app.get("/refresh")
    def refresh(authorization: str | None = Header(default=None)):
        if not authorization:
            raise HTTPException(401, "missing token")
        try:
            return svc.refresh(authorization.split(" ", 1)[-1])
        except Exception as e:
            raise HTTPException(401, str(e))

    @app.post("/logout")
    def logout():
        resp = JSONResponse({"status": "logged out"})
        resp.delete_cookie("auth_token")
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
        return {k: claims.get(k) for k in ("sub", "email", "name", "roles", "provider")}

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

    @app.get("/admin/role-assignments/pending", dependencies=[Depends(admin)])
    def pending():
        return {"pending": svc.roles.pending()}

    @app.get("/admin/users/search", dependencies=[Depends(admin)])
    def search(q: str):
        return {"users": svc.roles.search(q)}

    @app.get("/admin/users/{user_id}/roles", dependencies=[Depends(admin)])
    def get_roles(user_id: str):
        d = svc.roles.get(user_id)
        if d is None:
            raise HTTPException(404, "user not found")
        return {"user_id": user_id, "roles": d.get("roles", []), "status": d.get("status")}

    @app.post("/admin/users/{user_id}/roles", dependencies=[Depends(admin)])
    def assign(user_id: str, body: dict):
        try:
            return svc.roles.assign(user_id, body.get("roles", []))
        except KeyError:
            raise HTTPException(404, "user not found")

    @app.delete("/admin/users/{user_id}/roles", dependencies=[Depends(admin)])
    def revoke(user_id: str, body: dict):
        try:
            return svc.roles.revoke(user_id, body.get("roles", []))
        except KeyError:
            raise HTTPException(404, "user not found")

    @app.post("/admin/users/{user_id}/deny", dependencies=[Depends(admin)])
    def deny(user_id: str):
        return svc.roles.deny(user_id)

    return app
