#!/bin/bash
# __graft_entry__.smoke() on the GPU box
python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
