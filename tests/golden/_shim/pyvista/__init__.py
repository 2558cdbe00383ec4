"""Empty stand-in: pyvista is used only by render paths of the reference (never by step()). Fixture generation only."""
