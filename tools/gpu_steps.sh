#!/bin/bash
# Run GPU steps in order; stop at the first step that did not end with a pytest-style
# pass/fail (rc 0/1): faults, aborts, timeouts end the call.
for step in "$@"; do
  echo "=== $step"
  bash -c "$step"
  rc=$?
  echo "=== rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after rc=$rc"; exit $rc; fi
done
