"""Bearer-token acquisition for IAP-protected pipeline endpoints.

Reference: `sdk/python/kfp/_auth.py:28-109` (google-auth service-account JWT exchanged for a Google
OpenID Connect token with `target_audience=client_id`). Order here: `MIFX_KFP_TOKEN` env var ->
google-auth (if importable) -> `gcloud auth print-identity-token`; None if nothing is available."""
from __future__ import annotations

import logging
import os
import shutil
import subprocess

IAM_SCOPE = "https://www.googleapis.com/auth/iam"
OAUTH_TOKEN_URI = "https://www.googleapis.com/oauth2/v4/token"


def _google_auth_token(client_id: str) -> str | None:
    try:
        import google.auth  # type: ignore
        import google.auth.transport.requests  # type: ignore
        import google.oauth2.id_token  # type: ignore
    except ImportError:
        return None
    try:
        return google.oauth2.id_token.fetch_id_token(google.auth.transport.requests.Request(), client_id)
    except Exception as e:  # noqa: BLE001 - fall through to the next source
        logging.info("google-auth id token fetch failed: %s", e)
        return None


def _gcloud_token(client_id: str) -> str | None:
    if shutil.which("gcloud") is None:
        return None
    r = subprocess.run(["gcloud", "auth", "print-identity-token", f"--audiences={client_id}"],
                       capture_output=True, text=True)
    return r.stdout.strip() or None if r.returncode == 0 else None


def get_auth_token(client_id: str) -> str | None:
    tok = os.environ.get("MIFX_KFP_TOKEN")
    if tok:
        return tok
    return _google_auth_token(client_id) or _gcloud_token(client_id)
