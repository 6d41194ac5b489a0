"""Drop-in for the reference's moefication helpers (moefication/helper.py)."""
