"""CPU oracle of the traversal pass -- TEST INFRASTRUCTURE ONLY (see oracle.py)."""
