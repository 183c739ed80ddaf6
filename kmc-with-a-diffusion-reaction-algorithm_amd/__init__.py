"""MI355X-native engine for the KMC diffusion–reaction step loop."""
