"""`python -m haag_vq ...` = `vq-benchmark ...`."""

from .cli import main

main()
