"""Node runtime: API facade, HTTP handler, internal client, server wiring."""
