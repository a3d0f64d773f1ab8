import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libpinot_amd.so on the device)")


def pytest_sessionfinish(session, exitstatus):
    """Fail the session when any execution's partitioned self-check failed, even where a test swallowed the error:
    the library counts them process-wide (pinot_amd_selfcheck_failures). Sessions that never loaded the library
    (the CPU suite) are not touched."""
    if "pinot_amd._lib" not in sys.modules:
        return
    from pinot_amd import _lib
    if getattr(_lib, "_lib", None) is None:
        return
    from helpers import EXPECTED_SELFCHECK_FAILURES
    n = int(_lib.lib().pinot_amd_selfcheck_failures())
    if n != EXPECTED_SELFCHECK_FAILURES[0]:
        msg = (f"partitioned-plan self-check failures in this session: {n} "
               f"(expected {EXPECTED_SELFCHECK_FAILURES[0]} injected)")
        print("\n" + msg, file=sys.stderr)
        session.exitstatus = 1
    else:
        print(f"\npartitioned-plan self-check failures in this session: {n} (all injected by the suite)",
              file=sys.stderr)
