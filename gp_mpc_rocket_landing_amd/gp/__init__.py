"""GP surfaces (reference src/gp): kernels, exact / sparse GPs, features, structured GPs."""
