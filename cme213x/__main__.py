import sys

import cme213x  # noqa: F401  (installs the alias)
from cme213x.__main__ import main  # noqa: E402

sys.exit(main())
