#!/bin/bash
# round 4: the cadence sweep on the second corpus (all six cadences, 2 seeds, 2 single seeds)
bash profiles/r04/drivers/cadence2.sh 1024,2048,4096,8192,16384,30000 1,2 "" b
