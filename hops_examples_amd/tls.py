"""Certificate locations (``hops.tls``; notebooks/kafka/KafkaPython.ipynb:152-161).

Local services (kafka log, serving, jobs) run over loopback without TLS, so the
helpers return project-local paths under ``.certs/`` where a deployment would place
its CA chain / client certificate / key.  Nothing is generated and no secret is read.
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
