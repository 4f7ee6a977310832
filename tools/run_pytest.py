"""pytest as a script (so tools/with_lib.py can run the tests against another library build)."""
import sys

import pytest

if __name__ == "__main__":
    sys.exit(pytest.main(sys.argv[1:]))
