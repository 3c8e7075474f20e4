# VGPR / SGPR / spills / scratch / occupancy per kernel instantiation of librtmi355x (compile-time,
# no GPU).  Usage: scripts/resources.sh [> profiles/rNN_resource_usage.txt]
make -s -C "$(dirname "$0")/../eraytracer_amd/csrc" resource-usage 2>&1 | python3 "$(dirname "$0")/resource_table.py"
