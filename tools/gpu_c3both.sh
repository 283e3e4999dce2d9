#!/bin/bash
bash tools/gpu_c3w.sh && bash tools/gpu_c3diag.sh
