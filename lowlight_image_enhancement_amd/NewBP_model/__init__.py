"""NewBP_model API (reference: NewBP_model/)."""
