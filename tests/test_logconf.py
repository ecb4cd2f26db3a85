"""Logging layout (reference: config/log4j_{master,slave}.properties): stdout + daily-rolling
<role>.log (DEBUG+), <role>_warn.log (WARN+), <role>_error.log (ERROR+), or a logging.config file."""
import io
import logging
import os

from mp4x.utils.logconf import configure_logging

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _flush():
    for h in logging.getLogger().handlers:
        h.flush()


def test_threshold_split_files(tmp_path):
    buf = io.StringIO()
    configure_logging("master", log_dir=str(tmp_path), level="DEBUG", stream=buf)
    try:
        lg = logging.getLogger("mp4x.test")
        lg.debug("d-msg")
        lg.info("i-msg")
        lg.warning("w-msg")
        lg.error("e-msg")
        _flush()
        main = (tmp_path / "master.log").read_text()
        warn = (tmp_path / "master_warn.log").read_text()
        err = (tmp_path / "master_error.log").read_text()
        assert all(m in main for m in ("d-msg", "i-msg", "w-msg", "e-msg"))
        assert "w-msg" in warn and "e-msg" in warn and "i-msg" not in warn
        assert "e-msg" in err and "w-msg" not in err
        # log4j pattern: date, padded level, logger:line - message
        assert " ERROR mp4x.test:" in err and " - e-msg" in err
        assert "i-msg" in buf.getvalue()
        # idempotent: a second call replaces (not duplicates) its own handlers
        n = len(logging.getLogger().handlers)
        configure_logging("master", log_dir=str(tmp_path), level="DEBUG", stream=buf)
        assert len(logging.getLogger().handlers) == n
    finally:
        configure_logging("x", log_dir="-", level="WARNING", stream=io.StringIO())


def test_ini_config_file(tmp_path, monkeypatch):
    monkeypatch.chdir(tmp_path)
    os.makedirs("log")
    root = logging.getLogger()
    saved = list(root.handlers), root.level
    try:
        configure_logging(config_file=os.path.join(ROOT, "config", "logging_slave.ini"))
        logging.getLogger("mp4x.x").warning("from-ini")
        _flush()
        assert "from-ini" in (tmp_path / "log" / "slave.log").read_text()
        assert "from-ini" in (tmp_path / "log" / "slave_warn.log").read_text()
        assert (tmp_path / "log" / "slave_error.log").read_text() == ""
    finally:
        for h in list(root.handlers):
            root.removeHandler(h)
            h.close()
        for h in saved[0]:
            root.addHandler(h)
        root.setLevel(saved[1])
