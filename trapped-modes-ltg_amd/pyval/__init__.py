"""Drop-in for the reference's synthetic known-answer harness (/root/reference/pyval/)."""
