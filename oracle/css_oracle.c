/* CSS oracle: filled in with the CSS path */
