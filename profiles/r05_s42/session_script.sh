#!/bin/bash
# round-5 session 42: the default bench on another box, final sources (box-to-box spread)
bash tools/gpu_session.sh "python -u bench.py"
