"""Exception types the reference notebooks import (``from hops.exceptions import
APIKeyFileNotFound, RestAPIError``, jobs-client/flink/jobs_flink_client.py:9)."""


class HopsxError(Exception):
    pass


class RestAPIError(HopsxError):
    """A service call failed (local services raise it with the same shape: message + status)."""

    def __init__(self, message: str = "", status: int | None = None):
        super().__init__(message)
        self.status = status


class APIKeyFileNotFound(HopsxError):
    pass


class UnkownSecretStorageError(HopsxError):
    pass


class CouldNotConvertDataframe(HopsxError):
    pass
