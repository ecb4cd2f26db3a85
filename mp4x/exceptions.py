"""Error types.

Mirrors the reference's single checked exception ``Mp4jException``
(/root/reference/src/main/java/com/fenbi/mp4j/exception/Mp4jException.java:30-46):
every public collective raises it for illegal arguments, transport failures
and remote aborts.  Native status codes (``hipError_t`` / RCCL results) are
mapped onto :class:`NativeError`, a subclass, so callers can keep catching a
single type.
"""


class Mp4jException(Exception):
    """Base error of the library (reference: ``Mp4jException``)."""


# Idiomatic alias for new code.
Mp4xError = Mp4jException


class RangeError(Mp4jException):
    """Illegal ``[from, to)`` / counts arguments (reference CommUtils checks)."""


class TransportError(Mp4jException):
    """A peer connection or the master connection failed."""


class NativeError(Mp4jException):
    """A HIP / RCCL call inside the native extension returned an error."""

    def __init__(self, where: str, code: int, msg: str = ""):
        super().__init__(f"{where}: native error {code} {msg}".rstrip())
        self.where = where
        self.code = code


class CommAborted(Mp4jException):
    """The job was aborted (another rank closed with a non-zero code)."""
