import sys

from pilosa_amd.cli.main import main

sys.exit(main())
