import sys

import msbfs  # noqa: F401  (registers the alias)
from msbfs.__main__ import main  # noqa: E402

sys.exit(main())
