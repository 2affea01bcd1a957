"""Shared helpers of the GPU tests."""
import os

import pytest


def class_missing(e):
    """mas_create refused a config (abi.MasError e).  A capacity class that is
    not compiled is a skip only when the library was narrowed on purpose
    (MAS_CLASSES set in the environment, as for a partial `build()`); any
    other refusal, or a missing class of the full build, fails the test."""
    msg = str(e)
    if 'no compiled capacity class' in msg and os.environ.get('MAS_CLASSES'):
        pytest.skip(msg)
    pytest.fail(f'mas_create refused the config: {msg}')
