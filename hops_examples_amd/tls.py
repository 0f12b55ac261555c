"""Certificate locations (``hops.tls``; notebooks/kafka/KafkaPython.ipynb:152-161).

Local services (kafka log, serving, jobs) run over loopback without TLS, so the
helpers return project-local paths under ``.certs/`` where a deployment would place
its CA chain / client certificate / key (no secret is read).  ``make_local_certs`` creates a throw-away
CA + server / client certificates for local TLS endpoints (two-way TLS of hive_server.HiveServer2).
"""
from __future__ import annotations

from pathlib import Path

from . import hdfs


def _certs() -> Path:
    d = Path(hdfs.project_path()) / ".certs"
    d.mkdir(parents=True, exist_ok=True)
    return d


def get_ca_chain_location() -> str:
    return str(_certs() / "ca_chain.pem")


def get_client_certificate_location() -> str:
    return str(_certs() / "client_cert.pem")


def get_client_key_location() -> str:
    return str(_certs() / "client_key.pem")


def get_key_store() -> str:
    return str(_certs() / "k_certificate")


def get_trust_store() -> str:
    return str(_certs() / "t_certificate")


def get_key_store_pwd() -> str:
    return ""


get_trust_store_pwd = get_key_store_pwd


def make_local_certs(directory: str | None = None, days: int = 2) -> dict:
    """Create a throw-away CA plus a server (CN/SAN 127.0.0.1) and a client certificate signed by it
    with the ``openssl`` CLI, for local TLS endpoints (hive_server.HiveServer2 with two-way TLS).
    Returns the PEM paths: ca, server_cert, server_key, client_cert, client_key, client_bundle
    (certificate + key in one file: the ``sslKeyStore`` of a JDBC URL)."""
    import subprocess
    import tempfile

    d = Path(directory) if directory else Path(tempfile.mkdtemp(prefix="hopsx-certs-"))
    d.mkdir(parents=True, exist_ok=True)

    def run(*args):
        subprocess.run(["openssl", *args], check=True, capture_output=True)

    run("req", "-x509", "-newkey", "rsa:2048", "-nodes", "-keyout", str(d / "ca.key"), "-out", str(d / "ca.pem"),
        "-days", str(days), "-subj", "/CN=hopsx-local-ca")
    ext = d / "san.ext"
    ext.write_text("subjectAltName=IP:127.0.0.1,DNS:localhost\n")
    for who in ("server", "client"):
        run("req", "-newkey", "rsa:2048", "-nodes", "-keyout", str(d / f"{who}.key"), "-out", str(d / f"{who}.csr"),
            "-subj", f"/CN={'127.0.0.1' if who == 'server' else 'hopsx-client'}")
        run("x509", "-req", "-in", str(d / f"{who}.csr"), "-CA", str(d / "ca.pem"), "-CAkey", str(d / "ca.key"),
            "-CAcreateserial", "-out", str(d / f"{who}.pem"), "-days", str(days), "-extfile", str(ext))
    (d / "client_bundle.pem").write_text((d / "client.pem").read_text() + (d / "client.key").read_text())
    return {"ca": str(d / "ca.pem"), "server_cert": str(d / "server.pem"), "server_key": str(d / "server.key"),
            "client_cert": str(d / "client.pem"), "client_key": str(d / "client.key"),
            "client_bundle": str(d / "client_bundle.pem")}
