"""Empty stand-in: pygame is used only by render/keymap paths of the reference (never by step()). Fixture generation only."""
