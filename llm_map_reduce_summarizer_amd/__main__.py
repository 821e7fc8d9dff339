from .cli import main
from .parallel.dist import exit_process

# the bench's exit path (parallel/dist.py exit_process): a finished multi-rank job exits with its own code
exit_process(main())
