"""metrics API subset on the hot path (reference: metrics/)."""
