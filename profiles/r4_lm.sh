#!/bin/bash
bash profiles/r4_l.sh
bash profiles/r4_m.sh
