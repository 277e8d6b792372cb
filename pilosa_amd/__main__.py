"""python -m pilosa_amd -> CLI (reference cmd/pilosa/main.go)."""
import sys

from pilosa_amd.cli.main import main

if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
