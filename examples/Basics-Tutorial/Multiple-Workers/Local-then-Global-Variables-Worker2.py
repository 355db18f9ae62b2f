"""Worker 2 of the shared-PS-variable tutorial (see _worker.py)."""
from _worker import run

if __name__ == '__main__':
    run(1)
