import sys

from .jobs import main

sys.exit(main())
